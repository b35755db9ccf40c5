"""Trajectory rollouts (macm_world_rollout_traj / _bots_traj, macm_tdm_rollout_traj / _bots_traj):
K steps in one launch that keep every step's outputs, as the reference returns (obs, rewards) from
every env.step (gym_macm/envs/mvmnt.py:140; TDM: obs every step, combat.py:184).

The bar: row k of every [K, ...] output equals what step k of K per-step calls returned, bit for
bit; the state and counters after the rollout equal the per-step path's; the closed-loop form keeps
every step's bot actions (row k + 1 = bots.flock / bots.combat of step k's observation)."""
import numpy as np
import pytest
import torch

from test_gpu_rollout import assert_same, flock_actions

pytestmark = pytest.mark.gpu

from gym_macm.bots import combat_actions  # noqa: E402
from gym_macm.bots import flock_actions as bot_flock  # noqa: E402
from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402

KEYS = ("obs", "nbr_id", "reward", "collided", "done")


def per_step(vec, acts):
    rows = {k: [] for k in KEYS}
    for k in range(acts.shape[0]):
        vec.step(acts[k])
        for key in KEYS:
            rows[key].append(getattr(vec.world, key).clone())
    return {k: torch.stack(v) for k, v in rows.items()}


def assert_traj(ref, traj, ctx):
    for k in ref:
        assert traj[k].shape == ref[k].shape, f"{ctx}: {k} shape"
        assert torch.equal(traj[k], ref[k]), f"{ctx}: {k} (first differing step " \
            f"{int((traj[k] != ref[k]).reshape(ref[k].shape[0], -1).any(1).nonzero()[0])})"


@pytest.mark.parametrize("E,N,K,kw", [
    (64, 64, 9, {}),
    (48, 20, 8, {"obs_dtype": torch.float64, "coord": "cartesian"}),
    (40, 30, 6, {"action_mode": "continuous"}),
    (8, 64, 10, {"start_spread": 4}),  # dense: the spill step inside the loop
    (2100, 64, 4, {}),                 # >= 2048 envs: the headline's scalar-sweep instantiation
    (6, 100, 5, {"start_spread": 12}),  # workgroup path: three launches per step
    (1031, 100, 4, {"start_spread": 12}),  # workgroup path in env slices on their own streams
    (200, 64, 33, {}),                 # >= 32 steps: the envs in the balanced order (rollout_sched)
])
def test_flock_trajectory_equals_per_step(E, N, K, kw):
    cont = kw.get("action_mode") == "continuous"
    a = FlockVec(E, n_agents=[N], seed=5, device="cuda:0", **kw)
    b = FlockVec(E, n_agents=[N], seed=5, device="cuda:0", **kw)
    acts = flock_actions(K, E, N, 13, cont)
    ref = per_step(a, acts)
    traj = b.rollout(acts, trajectory=True)
    assert_traj(ref, traj, "trajectory")
    assert_same(a, b, "after the trajectory rollout")  # state, counters, the world's current outputs
    # into caller buffers, twice (the second starts from the first's list parity)
    buf = b.world.trajectory_buffers(K)
    acts2 = flock_actions(K, E, N, 14, cont)
    ref2 = per_step(a, acts2)
    b.rollout(acts2, trajectory=True, traj=buf)
    assert_traj(ref2, buf, "second trajectory")
    assert_same(a, b, "after the second trajectory rollout")


@pytest.mark.parametrize("E,N,K,kw", [
    (64, 64, 12, {}),
    (32, 20, 8, {"obs_dtype": torch.float64}),
    (4, 100, 4, {"start_spread": 12}),
    (1031, 100, 3, {"start_spread": 12}),
    (128, 64, 32, {}),  # the balanced order
])
def test_flock_closed_loop_trajectory(E, N, K, kw):
    a = FlockVec(E, n_agents=[N], seed=12, device="cuda:0", start_spread=kw.pop("start_spread", 6), **kw)
    b = FlockVec(E, n_agents=[N], seed=12, device="cuda:0", start_spread=a.settings.start_spread, **kw)
    act = bot_flock(a.obs)
    acts_b = torch.empty((K + 1, E, N, 3), dtype=torch.uint8, device="cuda:0")
    acts_b[0] = act
    rows_a = [act.clone()]
    ref = {k: [] for k in KEYS}
    for _ in range(K):
        a.step(act)
        for key in KEYS:
            ref[key].append(getattr(a.world, key).clone())
        bot_flock(a.obs, out=act)
        rows_a.append(act.clone())
    ref = {k: torch.stack(v) for k, v in ref.items()}
    traj = b.rollout_bots(acts_b, K, trajectory=True)
    assert_traj(ref, traj, "closed-loop trajectory")
    assert torch.equal(acts_b, torch.stack(rows_a)), "every step's bot actions"
    assert_same(a, b, "after the closed-loop trajectory")


def tdm_pair(teams, E, obs_f64=False):
    a = TdmWorld(tdm_config(teams, obs_f64=obs_f64), E, device="cuda:0")
    b = TdmWorld(tdm_config(teams, obs_f64=obs_f64), E, device="cuda:0")
    a.reset(7, 0)
    b.reset(7, 0)
    return a, b


TKEYS = TdmWorld._TRAJ_KEYS


def assert_tdm_state(a, b):
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=f"state[{k}]")
    np.testing.assert_array_equal(a.counters(), b.counters())


@pytest.mark.parametrize("teams,K,obs_f64", [([16, 16], 9, False), ([8, 8, 8], 10, True), ([16, 16], 32, False)])
def test_tdm_trajectory_equals_per_step(teams, K, obs_f64):
    E, N = 48, sum(teams)
    a, b = tdm_pair(teams, E, obs_f64)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(2)
    acts = torch.randint(0, 3, (K, E, N, 4), dtype=torch.uint8, device="cuda:0", generator=g)
    acts[..., 3] = torch.randint(0, 2, (K, E, N), dtype=torch.uint8, device="cuda:0", generator=g)
    ref = {k: [] for k in TKEYS}
    for k in range(K):
        a.step(acts[k])
        for key, t in zip(TKEYS, a.outputs()):
            ref[key].append(t.clone())
    ref = {k: torch.stack(v) for k, v in ref.items()}
    traj = b.rollout_traj(acts)
    assert_traj(ref, traj, "TDM trajectory")
    assert_tdm_state(a, b)
    assert int(a.counters()[1]) > 0


def test_tdm_closed_loop_trajectory():
    E, teams, K = 32, [8, 8], 30
    a, b = tdm_pair(teams, E)
    act = combat_actions(a.obs, a.mask)
    acts_b = torch.empty((K + 1, E, 16, 4), dtype=torch.uint8, device="cuda:0")
    acts_b[0] = act
    rows_a = [act.clone()]
    ref = {k: [] for k in TKEYS}
    for _ in range(K):
        a.step(act)
        for key, t in zip(TKEYS, a.outputs()):
            ref[key].append(t.clone())
        combat_actions(a.obs, a.mask, out=act)
        rows_a.append(act.clone())
    ref = {k: torch.stack(v) for k, v in ref.items()}
    traj = b.rollout_bots_traj(acts_b, K)
    assert_traj(ref, traj, "TDM closed-loop trajectory")
    assert torch.equal(acts_b, torch.stack(rows_a))
    assert_tdm_state(a, b)


def test_trajectory_argument_checks():
    v = FlockVec(4, n_agents=[16], seed=2, device="cuda:0")
    acts = flock_actions(3, 4, 16, 9)
    with pytest.raises(ValueError):
        v.rollout(acts, trajectory=True, traj=v.world.trajectory_buffers(2))  # too few rows
    with pytest.raises(ValueError):
        v.rollout_bots(torch.zeros((3, 4, 16, 3), dtype=torch.uint8, device="cuda:0"), 3, trajectory=True)
    out = v.rollout(acts[:0], trajectory=True)  # K = 0: nothing is stepped
    assert out["reward"].shape == (0, 4, 16)


def test_trajectory_buffers_are_checked_before_the_launch():
    """a caller buffer of the wrong dtype, env or agent count is refused (ValueError)
    before any kernel writes into it, for Flock and TDM."""
    E, N, K = 8, 16, 3
    v = FlockVec(E, n_agents=[N], seed=1, device="cuda:0")
    acts = flock_actions(K, E, N, 3, False)
    good = v.world.trajectory_buffers(K)
    bad = [dict(good, obs=good["obs"].double()),                        # f64 obs in an f32 world
           dict(good, reward=torch.empty((K, E - 1, N), device="cuda:0")),  # fewer envs
           dict(good, nbr_id=torch.empty((K, E, N - 1), dtype=torch.int32, device="cuda:0")),
           dict(good, done=torch.empty((K - 1, E), dtype=torch.uint8, device="cuda:0")),  # fewer steps
           dict(good, extra=good["done"])]
    for t in bad:
        with pytest.raises(ValueError):
            v.world.rollout_traj(acts, t)
    v.world.rollout_traj(acts, good)  # the right buffers still work
    w = TdmWorld(tdm_config([4, 4]), E, device="cuda:0")
    w.reset(2, 0)
    ta = torch.randint(0, 2, (K, E, 8, 4), dtype=torch.uint8, device="cuda:0")
    tg = w.trajectory_buffers(K)
    for t in (dict(tg, health=tg["health"].float()), dict(tg, obs=torch.empty((K, E, 8, 8, 4), device="cuda:0")),
              dict(tg, winner=tg["winner"].to(torch.int64))):
        with pytest.raises(ValueError):
            w.rollout_traj(ta, t)
    w.rollout_traj(ta, tg)


def test_raw_trajectory_launch_forms_agree():
    """bench.py's timed launch: rollout_traj_launcher (ctypes arguments and the outputs struct built
    before the timed region) writes what rollout_traj_raw and the checked rollout write."""
    E, N, K = 96, 64, 7
    a = FlockVec(E, n_agents=[N], seed=21, device="cuda:0")
    b = FlockVec(E, n_agents=[N], seed=21, device="cuda:0")
    c = FlockVec(E, n_agents=[N], seed=21, device="cuda:0")
    acts = flock_actions(K, E, N, 17)
    ref = a.rollout(acts, trajectory=True)
    sh = torch.cuda.current_stream().cuda_stream
    buf_b = b.world.trajectory_buffers(K)
    b.world.rollout_traj_raw(acts.data_ptr(), K, buf_b, sh)
    buf_c = c.world.trajectory_buffers(K)
    go = c.world.rollout_traj_launcher(acts.data_ptr(), K, c.world.traj_outputs(buf_c), sh)
    go()
    torch.cuda.synchronize()
    assert_traj(ref, buf_b, "rollout_traj_raw")
    assert_traj(ref, buf_c, "rollout_traj_launcher")
    for v in (b, c):
        sa, sv = a.world.get_state(), v.world.get_state()
        for k in sa:
            np.testing.assert_array_equal(sa[k], sv[k], err_msg=f"state[{k}]")


def test_raw_tdm_trajectory_launch_forms_agree():
    E, teams, K = 40, [16, 16], 6
    a, b = tdm_pair(teams, E)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(4)
    acts = torch.randint(0, 3, (K, E, 32, 4), dtype=torch.uint8, device="cuda:0", generator=g)
    ref = a.rollout_traj(acts)
    buf = b.trajectory_buffers(K)
    go = b.rollout_traj_launcher(acts.data_ptr(), K, b.traj_outputs(buf), torch.cuda.current_stream().cuda_stream)
    go()
    torch.cuda.synchronize()
    assert_traj(ref, buf, "TDM rollout_traj_launcher")
    assert_tdm_state(a, b)
