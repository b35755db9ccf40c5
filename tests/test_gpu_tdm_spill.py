"""TDM's spill step: crowded TDM envs bit-exact against the oracle.

The TDM wave kernel keeps its touching contacts in LDS (256 per env, 16 per body). An env beyond
either cap used to raise MACM_E_OVERFLOW; it now takes the spill step (csrc/flock_spill.hpp, MODE
kTdm) inside the same launch, after the wave kernel has taken the step's actions, melee ray casts
and deaths (combat.py:117-165): the spill step does the physics of the living bodies with an HBM
working set and TDM's env layer (observation, done / winner, counters). Bar: every state field, the
health / alive / done / winner / mask outputs and the observation equal the oracle's (oracle/,
the C restatement of combat.py over b2lite) at every step, status 0, and the spill step must
actually have run (macm_tdm_spilled)."""
import numpy as np
import pytest
import torch

from parity import combat_bot
from test_gpu_tdm import assert_tdm_state_equal, check_obs, check_rollout, make_pair, random_actions

pytestmark = pytest.mark.gpu

from gym_macm import _abi  # noqa: E402


@pytest.mark.parametrize("teams,side,seed,steps", [([32, 32], 5.0, 7, 100), ([32, 32], 3.0, 5, 60),
                                                   ([16, 16, 16, 16], 4.0, 9, 80)])
def test_tdm_crowded_world_spills_bit_exact(teams, side, seed, steps):
    """64 agents spawned in a side x side world: 269+ touching contacts (5 x 5) up to every body
    touching ~20 others (3 x 3), beyond the wave kernel's caps in the first steps."""
    E, N = 4, sum(teams)
    w, orc = make_pair(E, teams, seed=seed, world_width=side, world_height=side)
    rng = np.random.default_rng(seed)
    check_rollout(w, orc, steps, lambda o, m: random_actions(rng, E, N, p_attack=0.3), state_every=5)
    assert w.status() == 0
    assert w.spilled() > 0, "the crowded start never reached the spill step"


def test_tdm_2x16_in_6x6_world_100_steps():
    """TDM 2 x 16 in a 6 x 6 world, 100 steps, bit-exact (the wave kernel holds it:
    at most ~55 touching contacts, degree 8, oracle measurement)."""
    E, N = 16, 32
    w, orc = make_pair(E, [16, 16], seed=66, world_width=6.0, world_height=6.0)
    rng = np.random.default_rng(66)
    check_rollout(w, orc, 100, lambda o, m: random_actions(rng, E, N), state_every=5)


@pytest.mark.parametrize("teams,kw,policy", [
    ([16, 16], {}, "bot"),
    ([10, 10], dict(world_width=14.0, world_height=14.0), "random"),
    ([8, 8], dict(fresh_raycast=True, decay_mov_penalty=True, world_width=10.0, world_height=10.0), "bot"),
    ([16, 16, 16, 16], dict(obs_f64=True), "bot"),
])
def test_tdm_forced_spill_matches_oracle(teams, kw, policy):
    """Every env through the spill step (MACM_DEBUG_FORCE_SPILL) at ordinary densities, the settings
    variants included: deaths, the literal and the fresh listener, the decaying penalty, f64 obs."""
    E, N = 6, sum(teams)
    w, orc = make_pair(E, teams, seed=N + 3, **kw)
    w.set_debug(_abi.DEBUG_FORCE_SPILL)
    rng = np.random.default_rng(N)
    pol = combat_bot if policy == "bot" else (lambda o, m: random_actions(rng, E, N))
    steps = 150
    r = check_rollout(w, orc, steps, pol, state_every=10)
    assert w.spilled() == steps * E
    if policy == "bot":
        assert (r["alive"] == 0).any(), "no death in the forced-spill run"


def test_tdm_spill_pool_takes_turns():
    """Fewer working-set slots than crowded envs (the pooled form of a tight memory budget): the
    envs take the slots in turn, results stay bit-exact, no env is left unstepped."""
    E = 8
    w, orc = make_pair(E, [32, 32], seed=21, world_width=4.0, world_height=4.0)
    w.set_debug(_abi.DEBUG_SPILL_POOL | (2 << 8))
    rng = np.random.default_rng(21)
    check_rollout(w, orc, 25, lambda o, m: random_actions(rng, E, 64), state_every=5)
    assert w.status() == 0
    assert w.spilled() >= E


def test_tdm_rollout_launch_spills_bit_exact():
    """The multi-step TDM kernel (macm_tdm_rollout, its own translation unit) with crowded envs:
    K steps in one launch equal K oracle steps."""
    E, N, K = 4, 64, 40
    w, orc = make_pair(E, [32, 32], seed=3, world_width=4.0, world_height=4.0)
    rng = np.random.default_rng(3)
    acts = np.stack([random_actions(rng, E, N, p_attack=0.3) for _ in range(K)])
    w.rollout(torch.from_numpy(acts).cuda())
    for k in range(K):
        r = orc.step(acts[k])
    torch.cuda.synchronize()
    assert w.status() == 0 and w.spilled() > 0
    assert_tdm_state_equal(w.get_state(), orc.get_state(), "after the rollout launch")
    np.testing.assert_array_equal(w.health.cpu().numpy(), r["health"])
    np.testing.assert_array_equal(w.alive.cpu().numpy(), r["alive"])
    np.testing.assert_array_equal(w.mask.cpu().numpy(), r["mask"])
    check_obs(w, r["obs"], r["mask"], "rollout")
    np.testing.assert_array_equal(w.done.cpu().numpy(), r["done"])
    np.testing.assert_array_equal(w.winner.cpu().numpy(), r["winner"])
