"""macm_world_rollout / macm_tdm_rollout: K steps of every env with actions given in advance in
one launch (include/macm.h). The bar is the per-step path's: a rollout leaves exactly the state,
outputs and counters that K macm_world_step calls with the same actions leave (and so the
oracle's), for both parities of K, both observation widths, continuous actions, the spill step
inside the loop (dense worlds), the workgroup path (a launch sequence per step) and TDM.
Reference: the random-action loop `env.step(env.action_space.sample())` (mvmnt.py:271-293)."""
import numpy as np
import pytest
import torch

from parity import assert_state_equal
from test_gpu_parity import make_pair

pytestmark = pytest.mark.gpu

from gym_macm import _abi  # noqa: E402
from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402


def flock_actions(K, E, N, seed, continuous=False):
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    if continuous:
        return torch.rand((K, E, N, 2), device="cuda:0", generator=g) * 2 - 1
    return torch.randint(0, 3, (K, E, N, 3), dtype=torch.uint8, device="cuda:0", generator=g)


def outputs(w):
    return [t.clone() for t in (w.obs, w.nbr_id, w.reward, w.collided, w.done)]


def assert_same(a_vec, b_vec, ctx):
    for x, y, nm in zip(outputs(a_vec.world), outputs(b_vec.world), ("obs", "nbr", "reward", "collided", "done")):
        assert torch.equal(x, y), f"{ctx}: {nm}"
    sa, sb = a_vec.get_state(), b_vec.get_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=f"{ctx}: state[{k}]")
    np.testing.assert_array_equal(a_vec.counters(), b_vec.counters(), err_msg=f"{ctx}: counters")


@pytest.mark.parametrize("E,N,K,kw", [
    (64, 64, 7, {}),                                   # odd K: the list parity flips
    (64, 64, 10, {}),
    (48, 20, 9, {}),                                   # the 32-lane instantiation
    (32, 64, 6, {"obs_dtype": torch.float64}),
    (40, 30, 8, {"action_mode": "continuous"}),
    (8, 64, 12, {"start_spread": 4}),                  # dense: the spill step inside the loop
    (2100, 64, 5, {}),                                 # >= 2048 envs: the scalar-sweep instantiation
])
def test_flock_rollout_equals_per_step(E, N, K, kw):
    cont = kw.get("action_mode") == "continuous"
    a = FlockVec(E, n_agents=[N], seed=5, device="cuda:0", **kw)
    b = FlockVec(E, n_agents=[N], seed=5, device="cuda:0", **kw)
    acts = flock_actions(2 * K + 3, E, N, 11, cont)
    for k in range(K):
        a.step(acts[k])
    b.rollout(acts[:K])
    assert_same(a, b, f"after rollout of {K}")
    # stepping on after the rollout (one step, then a second rollout) stays in lockstep
    a.step(acts[K])
    b.step(acts[K])
    for k in range(K + 1, 2 * K + 3):
        a.step(acts[k])
    b.rollout(acts[K + 1:2 * K + 3])
    assert_same(a, b, "after step + second rollout")
    assert a.status() == 0 and b.status() == 0
    if kw.get("start_spread") == 4:
        assert b.spilled() > 0, "the dense start never reached the spill step"


def test_flock_rollout_matches_oracle():
    """40 steps of 16 envs x 64 agents in one launch against the oracle stepped 40 times."""
    E, N, K = 16, 64, 40
    vec, orc = make_pair(E, [N], seed=21, start_spread=8)
    rng = np.random.default_rng(3)
    acts = rng.integers(0, 3, size=(K, E, N, 3)).astype(np.uint8)
    vec.rollout(torch.from_numpy(acts).cuda())
    for k in range(K):
        r = orc.step(acts[k])
    assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), "rollout end")
    np.testing.assert_array_equal(vec.nbr_id.cpu().numpy(), r["nbr_id"])
    np.testing.assert_array_equal(vec.world.reward.cpu().numpy(), r["reward"].astype(np.float32))
    np.testing.assert_array_equal(vec.world.collided.cpu().numpy(), r["collided"])
    assert vec.status() == 0


def test_workgroup_path_rollout_equals_per_step():
    """N > 64: macm_world_rollout launches the split step K times."""
    E, N, K = 6, 100, 5
    a = FlockVec(E, n_agents=[N], seed=8, device="cuda:0", start_spread=12)
    b = FlockVec(E, n_agents=[N], seed=8, device="cuda:0", start_spread=12)
    acts = flock_actions(K, E, N, 4)
    for k in range(K):
        a.step(acts[k])
    b.rollout(acts)
    assert_same(a, b, "workgroup rollout")


@pytest.mark.parametrize("K", [4, 5])
def test_workgroup_path_sliced_rollout_equals_per_step(K):
    """>= 1024 envs on the workgroup path (N < 512): the rollout runs env slices on streams of
    their own with no join between steps (uneven slices: 1031 envs); twice, so the second rollout
    starts from the first one's list parity."""
    E, N = 1031, 100
    a = FlockVec(E, n_agents=[N], seed=8, device="cuda:0", start_spread=12)
    b = FlockVec(E, n_agents=[N], seed=8, device="cuda:0", start_spread=12)
    acts = flock_actions(2 * K, E, N, 6)
    for k in range(K):
        a.step(acts[k])
    b.rollout(acts[:K])
    assert_same(a, b, "sliced rollout")
    for k in range(K, 2 * K):
        a.step(acts[k])
    b.rollout(acts[K:])
    assert_same(a, b, "second sliced rollout")
    assert b.status() == 0


def test_rollout_zero_steps_and_validation():
    E, N = 4, 16
    v = FlockVec(E, n_agents=[N], seed=2, device="cuda:0", validate_actions=True)
    s0 = v.get_state()
    acts = flock_actions(3, E, N, 9)
    v.rollout(acts[:0])  # n_steps = 0: nothing happens
    acts[2, 1, 5, 0] = 3  # out of MultiDiscrete([3, 3, 3]) in the last step: no env is stepped
    with pytest.raises(_abi.MacmInvalidActionError):
        v.rollout(acts)
    s1 = v.get_state()
    for k in s0:
        np.testing.assert_array_equal(s0[k], s1[k], err_msg=k)
    with pytest.raises(ValueError):
        v.rollout(acts[0])  # not [K, E, N, 3]


@pytest.mark.parametrize("teams,K,obs_f64", [([16, 16], 9, False), ([8, 8, 8], 12, True)])
def test_tdm_rollout_equals_per_step(teams, K, obs_f64):
    E = 64
    N = sum(teams)
    a = TdmWorld(tdm_config(teams, obs_f64=obs_f64), E, device="cuda:0")
    b = TdmWorld(tdm_config(teams, obs_f64=obs_f64), E, device="cuda:0")
    a.reset(7, 0)
    b.reset(7, 0)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1)
    acts = torch.randint(0, 3, (K, E, N, 4), dtype=torch.uint8, device="cuda:0", generator=g)
    acts[..., 3] = torch.randint(0, 2, (K, E, N), dtype=torch.uint8, device="cuda:0", generator=g)
    for k in range(K):
        a.step(acts[k])
    b.rollout(acts)
    for x, y in zip(a.outputs(), b.outputs()):
        assert torch.equal(x, y)
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=f"state[{k}]")
    np.testing.assert_array_equal(a.counters(), b.counters())
    assert int(a.counters()[1]) > 0, "no melee attacks: the combat branch was not exercised"


@pytest.mark.parametrize("E,N,K,kw", [
    (64, 64, 9, {}),
    (32, 20, 8, {"obs_dtype": torch.float64, "coord": "cartesian"}),
    (4, 100, 4, {"start_spread": 12}),  # workgroup path: step + bots launches
    (1031, 100, 4, {"start_spread": 12}),  # workgroup path in env slices on their own streams
    (8, 100, 4, {"start_spread": 4}),  # dense: spill-stepped envs' next actions from kernel C too
    (6, 100, 3, {"start_spread": 12, "coord": "cartesian", "obs_dtype": torch.float64}),
])
def test_flock_closed_loop_rollout_equals_per_step(E, N, K, kw):
    """macm_world_rollout_bots vs K x (step, bots.flock) launches: same state, outputs and actions."""
    from gym_macm.bots import flock_actions
    a = FlockVec(E, n_agents=[N], seed=12, device="cuda:0", start_spread=kw.pop("start_spread", 6), **kw)
    b = FlockVec(E, n_agents=[N], seed=12, device="cuda:0", start_spread=a.settings.start_spread, **kw)
    act_a = flock_actions(a.obs)
    act_b = act_a.clone()
    for _ in range(K):
        a.step(act_a)
        flock_actions(a.obs, out=act_a)
    b.rollout_bots(act_b, K)
    assert_same(a, b, "closed-loop rollout")
    assert torch.equal(act_a, act_b), "the bot's next actions"


def test_tdm_closed_loop_rollout_equals_per_step():
    from gym_macm.bots import combat_actions
    E, teams, K = 32, [8, 8], 40
    a = TdmWorld(tdm_config(teams), E, device="cuda:0")
    b = TdmWorld(tdm_config(teams), E, device="cuda:0")
    a.reset(3, 0)
    b.reset(3, 0)
    act_a = combat_actions(a.obs, a.mask)
    act_b = act_a.clone()
    for _ in range(K):
        a.step(act_a)
        combat_actions(a.obs, a.mask, out=act_a)
    b.rollout_bots(act_b, K)
    for x, y in zip(a.outputs(), b.outputs()):
        assert torch.equal(x, y)
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=f"state[{k}]")
    assert torch.equal(act_a, act_b)
    assert int(a.counters()[1]) > 0


@pytest.mark.parametrize("E,N,K,kw", [
    (600, 64, 40, {"start_spread": 6}),                 # mixed densities: a non-trivial env order
    (300, 20, 33, {"obs_dtype": torch.float64}),        # the 32-lane instantiation, odd K
    (64, 64, 32, {"max_contacts": 50000}),              # beyond the order's 4096 buckets (200 KB of LDS unclamped)
])
def test_balanced_rollout_equals_per_step(E, N, K, kw):
    """Rollouts of >= 32 steps (kRollBalanceMinSteps) run env order[b] on wave b, the envs sorted by
    contact-list size (rollout_sched): open loop, then a closed loop, both against per-step launches."""
    from gym_macm.bots import flock_actions as bot_actions
    a = FlockVec(E, n_agents=[N], seed=17, device="cuda:0", **kw)
    b = FlockVec(E, n_agents=[N], seed=17, device="cuda:0", **kw)
    acts = flock_actions(K, E, N, 23)
    for k in range(K):
        a.step(acts[k])
    b.rollout(acts)
    assert_same(a, b, "balanced open-loop rollout")
    act_a = bot_actions(a.obs)
    act_b = act_a.clone()
    for _ in range(K):
        a.step(act_a)
        bot_actions(a.obs, out=act_a)
    b.rollout_bots(act_b, K)
    assert_same(a, b, "balanced closed-loop rollout")
    assert torch.equal(act_a, act_b), "the bot's next actions"
    assert b.status() == 0


@pytest.mark.parametrize("E,N,K,kw", [
    (40, 100, 12, {"start_spread": 12}),
    (24, 300, 8, {"reward_mode": "linear"}),
    (6, 1024, 6, {}),                                   # C5-shaped: dense DFS kernel, deep levels
    (1000, 256, 5, {"start_spread": 30}),               # >= 1024 envs would take the slices; 1000 do not
])
def test_handoff_equals_plain_workgroup_step(monkeypatch, E, N, K, kw):
    """The workgroup step's B -> C handoff (MACM_HANDOFF=1: kernel C on a second stream behind a watcher,
    taking the envs in kernel B's finish order, B's outputs handed over write-through) gives the plain
    launch order's results bit for bit: state, lists, outputs, counters and reward sums, per-step and
    rollout launches."""
    b = FlockVec(E, n_agents=[N], seed=E + N, device="cuda:0", **kw)
    a = FlockVec(E, n_agents=[N], seed=E + N, device="cuda:0", **kw)
    acts = flock_actions(2 * K, E, N, 7)
    for k in range(K):  # a world takes its handoff decision at its first workgroup step
        monkeypatch.setenv("MACM_HANDOFF", "0")
        a.step(acts[k])
        monkeypatch.setenv("MACM_HANDOFF", "1")
        b.step(acts[k])
    assert b.world.uses_handoff() and not a.world.uses_handoff()
    assert_same(a, b, "handoff per-step launches")
    for k in range(K, 2 * K):
        a.step(acts[k])
    b.rollout(acts[K:])
    assert_same(a, b, "handoff rollout")
    np.testing.assert_array_equal(a.counters(), b.counters())
    pa, ta = a.reward_sums()
    pb, tb = b.reward_sums()
    np.testing.assert_array_equal(pa, pb)
    assert ta == tb and b.status() == 0


def test_handoff_after_a_long_backlog_on_the_callers_stream(monkeypatch):
    """the handoff's watcher (kernel C's stream) must start its ~1 s clock only when kernel
    B's dependencies have finished, not when its own stream is idle. A > 1.5 s spin kernel queued on the
    caller's stream ahead of every handoff step (a PPO update between rollouts, say) must leave the
    steps' status 0 and their results equal to the plain launch order's."""
    import time
    E, N, K = 64, 100, 2
    monkeypatch.setenv("MACM_HANDOFF", "0")
    a = FlockVec(E, n_agents=[N], seed=41, device="cuda:0")
    monkeypatch.setenv("MACM_HANDOFF", "1")
    b = FlockVec(E, n_agents=[N], seed=41, device="cuda:0")
    acts = flock_actions(K, E, N, 23)
    # calibrate torch's spin kernel (its clock's rate is the device's) to ~2 s
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1000)
    e0.record()
    torch.cuda._sleep(10 ** 7)
    e1.record()
    torch.cuda.synchronize()
    cycles = int(10 ** 7 * 2000.0 / max(e0.elapsed_time(e1), 1e-3))
    for k in range(K):
        a.step(acts[k])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda._sleep(cycles)  # the backlog, on the stream the world steps on
        b.step(acts[k])
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 > 1.5, "the backlog kernel did not spin long enough to test this"
    assert b.world.uses_handoff()
    assert b.status() == 0, b.status()
    assert_same(a, b, "handoff behind a backlog")


def test_handoff_is_off_under_serialized_dispatch():
    """With kernel dispatches serialised (AMD_SERIALIZE_KERNEL, or a profiler collecting counters:
    ROCPROF_COUNTER_COLLECTION) the B -> C handoff's consumer cannot run beside its producer; the
    library then steps without it, and the results are complete and equal to the default run's."""
    import os
    import subprocess
    import sys
    code = r'''
import sys, numpy as np, torch
sys.path.insert(0, "gym-macm_amd")
from gym_macm.vec import FlockVec
E, N, K = 48, 100, 3
v = FlockVec(E, n_agents=[N], seed=9, device="cuda:0")
g = torch.Generator(device="cuda:0"); g.manual_seed(3)
for _ in range(K):
    v.step(torch.randint(0, 3, (E, N, 3), dtype=torch.uint8, device="cuda:0", generator=g))
torch.cuda.synchronize()
assert v.status() == 0, v.status()
c = v.counters()
assert int(c[0]) == E * N * K, c
np.save(sys.argv[1], v.get_state()["pos"])
'''
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for extra in ({"ROCPROF_COUNTER_COLLECTION": "1"}, {"AMD_SERIALIZE_KERNEL": "3"}, {}):
        env = dict(os.environ, MACM_HANDOFF="1", **extra)
        out = os.path.join(repo, "gpurun_out", f"serialized_{len(outs)}.npy")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        r = subprocess.run([sys.executable, "-c", code, out], cwd=repo, env=env, capture_output=True, text=True,
                           timeout=240)
        assert r.returncode == 0, (extra, r.stdout[-2000:], r.stderr[-2000:])
        outs.append(np.load(out))
    np.testing.assert_array_equal(outs[0], outs[2])
    np.testing.assert_array_equal(outs[1], outs[2])
