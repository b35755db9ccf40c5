"""Dense worlds: every valid reference configuration steps correctly, whatever its density.

The reference (Box2D) accepts any start_spread (gym_macm/settings.py:119-121,143-144 ->
envs/mvmnt.py:62-63); the fast kernels keep their per-contact arrays in LDS with fixed
capacities (wave kernel: 256 touching contacts, 16 per body; workgroup kernel A: 5 x blockDim
up to 4608). Envs beyond them take the spill step (csrc/flock_spill.hpp, HBM working set sized
by max_contacts) inside the same launch. Bar: bit-exact against the oracle for >= 100 steps with
status 0, and the spill step must actually have run (macm_world_spilled > 0).

Also here: the spill step forced for every env (MACM_DEBUG_FORCE_SPILL) at ordinary densities,
loud errors for what can still overflow (an explicit small max_contacts), set_state validation,
and the opt-in action validation (mvmnt.py:94 / combat.py:118). TDM's dense envs: test_gpu_tdm_spill.py."""
import random

import numpy as np
import pytest
import torch

from parity import assert_state_equal
from test_gpu_parity import check_rollout, make_pair, rand_actions

pytestmark = pytest.mark.gpu

from gym_macm import _abi  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402


@pytest.mark.parametrize("spread,seed", [(3, 31), (4, 41)])
def test_dense_64_agents_spill_bit_exact(spread, seed):
    """N = 64 at start_spread 3 / 4: up to ~540 / ~320 touching contacts and degree ~30 / ~18
    in the first steps (oracle measurement), beyond the wave kernel's 256 / 16."""
    vec, orc = make_pair(8, [64], seed=seed, start_spread=spread)
    check_rollout(vec, orc, 110, np.random.default_rng(seed), state_every=5)
    assert vec.status() == 0
    assert vec.spilled() > 0, "the dense start never reached the spill step"


def test_dense_256_agents_spread_8_spill_bit_exact():
    """N = 256 at start_spread 8: ~1500 touching contacts at the start, beyond kernel A's 1280."""
    vec, orc = make_pair(3, [256], seed=28, start_spread=8)
    check_rollout(vec, orc, 100, np.random.default_rng(8), state_every=10)
    assert vec.status() == 0
    assert vec.spilled() > 0


@pytest.mark.parametrize("E,N,spread,slots,steps", [(12, 64, 3, 2, 30), (3, 256, 8, 1, 12)])
def test_spill_pool_takes_turns(E, N, spread, slots, steps):
    """A world whose memory budget holds fewer spill working-set slots than envs (the
    working set was allocated for every env) shares a pool: dense envs take a slot for their spill
    step in turn (spill::acquire_slot). Forced here to 2 / 1 slots for 12 / 3 dense envs: results
    stay bit-exact and every env is stepped (no MACM_ST_SPILL_WAIT)."""
    vec, orc = make_pair(E, [N], seed=E + N, start_spread=spread)
    vec.world.set_debug(_abi.DEBUG_SPILL_POOL | (slots << 8))
    check_rollout(vec, orc, steps, np.random.default_rng(N), state_every=5)
    assert vec.status() == 0
    assert vec.spilled() >= E, "the envs never took the spill step"


def test_default_capacities_from_the_device_budget():
    """max_contacts = 0: every pair for N <= 64; one spill slot per env where the budget allows."""
    v = FlockVec(64, n_agents=[64], seed=1, device="cuda:0")
    assert v.world.C == 64 * 63 // 2 and v.world.spill_slots == 64
    w = FlockVec(8, n_agents=[1024], seed=1, device="cuda:0")
    assert w.world.C == 1024 * 1023 // 2 and w.world.spill_slots == 8  # 8 envs fit every pair


def test_c5_shaped_world_at_start_spread_5():
    """a C5-shaped env (1024 agents) at start_spread 5 (41 bodies per m^2: ~10^5
    fat-AABB pairs and tens of thousands of touching contacts per env) steps through the spill step
    with status 0 and the default capacity, bit-exact against the oracle."""
    vec, orc = make_pair(2, [1024], seed=5, start_spread=5)
    assert vec.world.C == 1024 * 1023 // 2
    check_rollout(vec, orc, 2, np.random.default_rng(5), state_every=1)
    assert vec.status() == 0 and vec.spilled() == 4


def test_dense_1024_agents_spread_14_spill():
    """N = 1024 at start_spread 14 (5.2 bodies per m^2): beyond kernel A's 4608 touching contacts."""
    vec, orc = make_pair(1, [1024], seed=14, start_spread=14)
    check_rollout(vec, orc, 8, np.random.default_rng(14), state_every=2)
    assert vec.spilled() > 0


@pytest.mark.parametrize("n_agents,kw", [
    ([4], dict(start_spread=3)),
    ([16], dict(start_spread=6, reward_mode="linear", coord="cartesian")),
    ([64], dict(start_spread=10)),
    ([40], dict(start_spread=8, action_mode="continuous")),
    ([100], dict(start_spread=12)),
    ([256], dict(start_spread=20, velocityIterations=3, positionIterations=1)),
])
def test_forced_spill_matches_oracle(n_agents, kw):
    """Every env through the spill step (test hook) at ordinary densities, both callers (the wave
    kernel for N <= 64, kernel A above), all settings variants: the spill step alone is bit-exact."""
    E = 4
    vec, orc = make_pair(E, n_agents, seed=sum(n_agents) + 5, **kw)
    vec.world.set_debug(_abi.DEBUG_FORCE_SPILL)
    N = vec.N
    rng = np.random.default_rng(N)
    fn = None
    if kw.get("action_mode") == "continuous":
        fn = lambda t: rng.uniform(-1.2, 1.2, size=(E, N, 2)).astype(np.float32)  # noqa: E731
    check_rollout(vec, orc, 60, rng, state_every=10, actions_fn=fn)
    assert vec.spilled() == 60 * E


def test_dropin_dict_api_dense_spread_4():
    """gym_macm.make(..., n_agents=[64], start_spread=4) through the dict API vs the oracle env
    constructed after the same random.seed (CPython MT19937 draws, mvmnt.py:47-64)."""
    from gym_macm.envs import Flock
    from oracle import OracleFlock
    seed, N = 4242, 64
    random.seed(seed)
    env = Flock(n_agents=[N], device="cuda:0", start_spread=4)
    orc = OracleFlock(to_config(flockSettings(start_spread=4), N, 1, obs_f64=True), None, 1, seed)
    rng = np.random.default_rng(1)
    for t in range(100):
        a = rand_actions(rng, 1, N)
        obs, rewards = env.step({i: a[0, i].astype(np.int64) for i in range(N)})
        r = orc.step(a)
        exp = [int(v) if v != -1 else -1 for v in r["reward"][0]]
        assert [rewards[i] for i in range(N)] == exp, f"rewards step {t}"
        np.testing.assert_array_equal([obs[i]["nodes"][0]["id"] for i in range(N)], r["nbr_id"][0],
                                      err_msg=f"nbr step {t}")
        got = np.array([np.concatenate([obs[i]["nodes"][0]["position"], obs[i]["nodes"][1]["position"]])
                        for i in range(N)])
        np.testing.assert_allclose(got, r["obs"][0], rtol=0, atol=1e-12, err_msg=f"obs step {t}")
    assert_state_equal(env.world.get_state(), orc.get_state(env.world.C), "dict api")
    assert env.world.spilled() > 0


# ---- what can still overflow is loud ------------------------------------------------------------


def test_contact_list_overflow_raises():
    """An explicit max_contacts below the fat-AABB pair count: the reset reports it and every
    later step refuses (MacmOverflowError, a MacmLibraryError) until the world is reset."""
    v = FlockVec(4, n_agents=[64], seed=3, device="cuda:0", start_spread=4, max_contacts=8)
    assert v.status() & _abi.ST_CONTACT_OVERFLOW
    a = torch.ones((4, 64, 3), dtype=torch.uint8, device="cuda:0")
    with pytest.raises(_abi.MacmOverflowError):
        v.step(a)
    with pytest.raises(_abi.MacmLibraryError):
        v.check_status()


def test_list_overflow_during_stepping_raises_on_next_step():
    """A list that fits at reset and outgrows max_contacts later (agents drawn together)."""
    E, N = 2, 100
    v = FlockVec(E, n_agents=[N], seed=9, device="cuda:0", start_spread=30, max_contacts=150)
    assert v.status() == 0
    st = v.get_state()
    st["pos"][:] = st["pos"] * np.float32(0.2)  # pack the bodies: far more overlapping pairs
    st["contact_count"][:] = 0
    v.set_state(st)
    a = torch.ones((E, N, 3), dtype=torch.uint8, device="cuda:0")
    v.step(a)
    torch.cuda.synchronize()
    with pytest.raises(_abi.MacmOverflowError):
        v.step(a)
    v.reset()
    v.step(a)  # a reset clears the condition


def test_reset_envs_clears_the_overflow_of_the_envs_it_resets():
    """reset_envs re-derives the host status word from the envs it did not reset. Env 1
    outgrows max_contacts; resetting env 0 only leaves the error, resetting env 1 clears it."""
    E, N = 2, 100
    v = FlockVec(E, n_agents=[N], seed=9, device="cuda:0", start_spread=30, max_contacts=150)
    st = v.get_state()
    st["pos"][1] = st["pos"][1] * np.float32(0.2)  # env 1 only: far more overlapping pairs
    st["contact_count"][:] = 0
    v.set_state(st)
    a = torch.ones((E, N, 3), dtype=torch.uint8, device="cuda:0")
    v.step(a)
    torch.cuda.synchronize()
    with pytest.raises(_abi.MacmOverflowError):
        v.step(a)
    v.reset_envs(torch.tensor([1, 0], dtype=torch.uint8, device="cuda:0"))
    with pytest.raises(_abi.MacmOverflowError):
        v.step(a)
    v.reset_envs(torch.tensor([0, 1], dtype=torch.uint8, device="cuda:0"))
    assert v.status() == 0
    v.step(a)  # the overflowed env was reset: stepping resumes


def test_set_state_rejects_invalid_lists():
    v = FlockVec(2, n_agents=[16], seed=1, device="cuda:0")
    good = v.get_state()
    bad = {k: x.copy() for k, x in good.items()}
    bad["contact_count"][0] = v.world.C + 1
    with pytest.raises(ValueError):
        v.set_state(bad)
    bad = {k: x.copy() for k, x in good.items()}
    bad["contact_count"][1] = 1
    bad["contact_ab"][1, 0] = 5 | (3 << 16)  # a > b
    with pytest.raises(_abi.MacmError):
        v.set_state(bad)
    bad["contact_ab"][1, 0] = 3 | (16 << 16)  # b = N
    with pytest.raises(_abi.MacmError):
        v.set_state(bad)
    v.set_state(good)  # still usable, state intact
    assert_state_equal(v.get_state(), good, "after rejected set_state")


def test_set_state_across_capacities():
    """A state saved from a world with another max_contacts loads when its lists fit."""
    E, N = 4, 100
    big, orc = make_pair(E, [N], seed=12, start_spread=15)
    rng = np.random.default_rng(0)
    for _ in range(20):
        a = rand_actions(rng, E, N)
        big.step(torch.from_numpy(a).cuda())
        orc.step(a)
    st = big.get_state()
    small = FlockVec(E, n_agents=[N], seed=0, device="cuda:0", start_spread=15,
                     max_contacts=int(st["contact_count"].max()) + 3)
    small.set_state(st)
    check_rollout(small, orc, 20, rng, state_every=5)


# ---- validate_actions (assert action_space.contains, mvmnt.py:94) ----------------------------------


def test_validate_actions_discrete():
    E, N = 3, 8
    v = FlockVec(E, n_agents=[N], seed=2, device="cuda:0", validate_actions=True)
    before = v.get_state()
    a = torch.ones((E, N, 3), dtype=torch.uint8, device="cuda:0")
    a[1, 5, 2] = 3
    with pytest.raises(_abi.MacmInvalidActionError, match="env 1 agent 5"):
        v.step(a)
    assert_state_equal(v.get_state(), before, "no env stepped")
    a8 = torch.ones((E, N, 3), dtype=torch.int8, device="cuda:0")
    a8[2, 0, 0] = -1
    with pytest.raises(_abi.MacmInvalidActionError, match="env 2 agent 0"):
        v.step(a8)
    a[1, 5, 2] = 2
    v.step(a)  # valid actions step normally
    assert int(v.get_state()["step_count"][0]) == 1


def test_validate_actions_continuous():
    E, N = 2, 6
    v = FlockVec(E, n_agents=[N], seed=2, device="cuda:0", validate_actions=True, action_mode="continuous")
    a = torch.zeros((E, N, 2), dtype=torch.float32, device="cuda:0")
    for bad in (float("nan"), 1.5, -1.0001):
        a[0, 3, 1] = bad
        with pytest.raises(_abi.MacmInvalidActionError, match="env 0 agent 3"):
            v.step(a)
    a[0, 3, 1] = -1.0
    v.step(a)


def test_validate_actions_tdm_ignores_dead_rows():
    from gym_macm.tdm_world import TdmWorld, tdm_config
    w = TdmWorld(tdm_config([2, 2], validate_actions=True), 2, device="cuda:0")
    w.reset(3)
    st = w.get_state()
    st["alive"][0, 1] = 0
    st["health"][0, 1] = 0.0
    w.set_state(st)
    a = torch.ones((2, 4, 4), dtype=torch.uint8, device="cuda:0")
    a[..., 3] = 0
    a[0, 1, 0] = 7  # a dead agent's row: not in the action space (combat.py:186-188), ignored
    w.step(a)
    a[1, 2, 3] = 2  # attack must be 0 or 1
    with pytest.raises(_abi.MacmInvalidActionError, match="env 1 agent 2"):
        w.step(a)
