"""Randomised configurations, HIP path vs the CPU oracle (same bar as
test_gpu_parity.py / test_gpu_tdm.py: bit-exact state, f32 obs within 1 ulp).

Every setting the C-ABI exposes is drawn from a seeded generator: agent counts on
both kernels (wave <= 64 < workgroup), hz, solver iterations (including 0),
warm starting, body radius/density/friction/damping, forces, rotation speed,
spawn spread, action/reward/coord modes, obs dtype; TDM team layouts, world
size, melee constants and the two literal-behaviour switches."""
import numpy as np
import pytest
import torch

from oracle import OracleTDM
from parity import combat_bot, flock_bot
from test_gpu_parity import check_rollout
from test_gpu_tdm import assert_tdm_state_equal, check_obs, random_actions

pytestmark = pytest.mark.gpu

from gym_macm.settings import CircleFixture, flockSettings, to_config  # noqa: E402
from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402
from parity import oracle_for  # noqa: E402


def flock_case(rng):
    N = int(rng.choice([2, 3, 7, 16, 31, 48, 64, 65, 90]))
    kw = dict(
        hz=float(rng.choice([30.0, 60.0, 120.0])),
        velocityIterations=int(rng.integers(0, 11)),
        positionIterations=int(rng.integers(0, 5)),
        enableWarmStarting=bool(rng.integers(0, 2)),
        start_spread=float(rng.uniform(4, 30)),
        agent_force=float(rng.choice([5, 20, 60])),
        agent_rotation_speed=float(rng.uniform(1, 8)),
        action_mode=str(rng.choice(["discrete", "continuous"])),
        reward_mode=str(rng.choice(["binary", "linear"])),
        coord=str(rng.choice(["polar", "cartesian"])),
        bodySettings={"fixtures": CircleFixture(float(rng.uniform(0.3, 0.8)), float(rng.uniform(0.5, 2.0)),
                                                float(rng.uniform(0.0, 1.0))),
                      "linearDamping": float(rng.uniform(0.0, 10.0)), "fixedRotation": True},
    )
    T = int(rng.integers(1, 4))
    targets = [int(i % T) for i in range(N)] if T > 1 else None
    return N, T, targets, kw


@pytest.mark.parametrize("case", range(12))
def test_flock_random_configs(case):
    rng = np.random.default_rng(1000 + case)
    N, T, targets, kw = flock_case(rng)
    E = 6
    f64 = bool(rng.integers(0, 2))
    vec = FlockVec(E, n_agents=[N], targets=targets, seed=case, device="cuda:0",
                   obs_dtype=torch.float64 if f64 else torch.float32, **kw)
    cfg = to_config(flockSettings(**kw), N, vec.n_targets, obs_f64=True)
    orc = oracle_for(cfg, vec.targets_idx, E, case)
    cont = kw["action_mode"] == "continuous"

    def acts(t):
        if cont:
            return rng.uniform(-1.2, 1.2, size=(E, N, 2)).astype(np.float32)
        if t % 3 == 2 and kw["coord"] == "polar":
            return flock_bot(orc.observe()[0])
        return rng.integers(0, 3, size=(E, N, 3)).astype(np.uint8)

    check_rollout(vec, orc, 40, rng, state_every=8, actions_fn=acts, obs_f64=f64)


def tdm_case(rng):
    nt = int(rng.integers(1, 5))
    sizes = [int(rng.integers(1, 64 // nt + 1)) for _ in range(nt)]
    if sum(sizes) < 2:
        sizes[0] = 2
    w = float(rng.uniform(6, 30))
    kw = dict(world_width=w, world_height=float(rng.uniform(6, 30)), hz=float(rng.choice([30.0, 60.0])),
              velocity_iterations=int(rng.integers(1, 10)), position_iterations=int(rng.integers(0, 4)),
              melee_range=float(rng.uniform(1, 4)), melee_dmg=float(rng.choice([0.1, 0.25, 0.5])),
              cooldown_atk=float(rng.uniform(0.2, 1.5)), cooldown_mov_penalty=float(rng.uniform(0.1, 1.0)),
              fresh_raycast=bool(rng.integers(0, 2)), decay_mov_penalty=bool(rng.integers(0, 2)))
    return sizes, kw


@pytest.mark.parametrize("case", range(8))
def test_tdm_random_configs(case):
    rng = np.random.default_rng(2000 + case)
    sizes, kw = tdm_case(rng)
    E, N = 6, sum(sizes)
    f64 = bool(rng.integers(0, 2))
    w = TdmWorld(tdm_config(sizes, obs_f64=f64, **kw), E, device="cuda:0")
    w.reset(case)
    orc = OracleTDM(tdm_config(sizes, obs_f64=True, **kw), E, case)
    obs, mask = orc.observe()
    for t in range(80):
        a = combat_bot(obs, mask) if t % 2 else random_actions(rng, E, N)
        w.step(torch.from_numpy(a).cuda())
        r = orc.step(a)
        obs, mask = r["obs"], r["mask"]
        np.testing.assert_array_equal(w.health.cpu().numpy(), r["health"], err_msg=f"health step {t}")
        np.testing.assert_array_equal(w.alive.cpu().numpy(), r["alive"], err_msg=f"alive step {t}")
        np.testing.assert_array_equal(w.winner.cpu().numpy(), r["winner"], err_msg=f"winner step {t}")
        np.testing.assert_array_equal(w.done.cpu().numpy(), r["done"], err_msg=f"done step {t}")
        check_obs(w, obs, mask, f"step {t}")
        if t % 10 == 9:
            assert_tdm_state_equal(w.get_state(), orc.get_state(), f"step {t}")
    assert w.status() == 0
