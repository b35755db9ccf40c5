"""The split TDM observation (round 6, csrc/tdm_obs_snap.hip): the wave kernel writes
pose snapshots and tdm_observe_snap observes every (step, env) row with a workgroup of its own. It
must give the fused form's outputs bit for bit (obs, mask, health, alive, done, winner, state,
counters) through every entry point that takes it: per-step launches, the overwrite rollout and the
trajectory rollout in chunks (K = 19: chunks of 8, 8 and 3 on two snapshot halves), float32 and
float64 observations, deaths, and envs that take the spill step (MACM_DEBUG_FORCE_SPILL). The fused
form itself is pinned to the oracle by test_gpu_tdm.py; the split form is the default below 1024 envs,
so those tests run it too. MACM_TDM_SPLIT_OBS=0/1 selects the form per call.

The tail observation (round 6, flock_step_w64.hip TailObs; the default for trajectory rollouts below
2048 envs): every env's wave steps its K steps writing write-through snapshots and publishing them, and
the finished waves plus observe-only waves observe the (step, env) rows from sub-queues; the same bits
as the fused form (test_tail_equals_fused; MACM_TDM_TAIL_OBS=0/1 and MACM_TDM_TAIL_WORKERS select)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from gym_macm import _abi  # noqa: E402
from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402


def actions(K, E, N, seed, p_attack=0.5):
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    a = torch.randint(0, 3, (K, E, N, 4), dtype=torch.uint8, device="cuda:0", generator=g)
    a[..., 3] = (torch.rand((K, E, N), device="cuda:0", generator=g) < p_attack).to(torch.uint8)
    return a


def same_outputs(a, b, ctx):
    for x, y, nm in zip(a.outputs(), b.outputs(), ("obs", "mask", "health", "alive", "done", "winner")):
        assert torch.equal(x, y), f"{ctx}: {nm}"


def same_state(a, b, ctx):
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=f"{ctx}: state[{k}]")
    np.testing.assert_array_equal(a.counters(), b.counters(), err_msg=f"{ctx}: counters")


def pair(monkeypatch, E, teams, seed, debug=0, **kw):
    ws = []
    for _ in range(2):
        w = TdmWorld(tdm_config(teams, **kw), E, device="cuda:0")
        if debug:
            w.set_debug(debug)
        w.reset(seed, 0)
        ws.append(w)
    return ws


def call(monkeypatch, split, fn, *args):
    monkeypatch.setenv("MACM_TDM_SPLIT_OBS", "1" if split else "0")
    r = fn(*args)
    monkeypatch.delenv("MACM_TDM_SPLIT_OBS")
    return r


@pytest.mark.parametrize("E,teams,kw,debug", [
    (512, [16, 16], {}, 0),                                   # BASELINE C4's per-GPU shard
    (37, [16, 16], {"obs_f64": True}, 0),
    (64, [3, 3, 3], {"fresh_raycast": True}, 0),
    (24, [32, 32], {}, 0),                                    # N = 64: the 64-lane instantiation
    (16, [8, 8], {"world_width": 8.0, "world_height": 8.0}, 0),   # crowded: deaths early
    (12, [16, 16], {}, _abi.DEBUG_FORCE_SPILL),               # every env through the spill step
])
def test_split_equals_fused(monkeypatch, E, teams, kw, debug):
    N = sum(teams)
    K = 19
    a, b = pair(monkeypatch, E, teams, 1000 + E + N, debug, **kw)
    acts = actions(3 * K + 2, E, N, E * N)
    for k in range(K):  # per-step launches
        call(monkeypatch, False, a.step, acts[k])
        call(monkeypatch, True, b.step, acts[k])
        same_outputs(a, b, f"step {k}")
    same_state(a, b, "per-step launches")
    ta = call(monkeypatch, False, a.rollout_traj, acts[K:2 * K])  # trajectory: chunks 8, 8, 3
    tb = call(monkeypatch, True, b.rollout_traj, acts[K:2 * K])
    for key in ta:
        assert torch.equal(ta[key], tb[key]), f"trajectory rollout: {key}"
    same_state(a, b, "trajectory rollout")
    call(monkeypatch, False, a.rollout, acts[2 * K:3 * K + 2])  # overwrite: the last step's outputs
    call(monkeypatch, True, b.rollout, acts[2 * K:3 * K + 2])
    same_outputs(a, b, "overwrite rollout")
    same_state(a, b, "overwrite rollout")
    assert a.status() == 0 and b.status() == 0
    if debug:
        assert b.spilled() > 0


def test_default_form_below_1024_envs(monkeypatch):
    """The launch form the library picks itself (the tail observation for trajectory rollouts below 1024
    envs) equals the forced fused form at 512 envs (C4's shard), in the trajectory rollout the
    benchmark times."""
    E, teams, K = 512, [16, 16], 20
    monkeypatch.delenv("MACM_TDM_SPLIT_OBS", raising=False)
    monkeypatch.delenv("MACM_TDM_TAIL_OBS", raising=False)
    a, b = pair(monkeypatch, E, teams, 77)
    assert b.launch_flags() & _abi.LAUNCH_TAIL_OBS
    acts = actions(K, E, 32, 5)
    ta = call_env(monkeypatch, FUSED, a.rollout_traj, acts)
    tb = b.rollout_traj(acts)  # default
    for key in ta:
        assert torch.equal(ta[key], tb[key]), key
    same_state(a, b, "default form")


def call_env(monkeypatch, env, fn, *args):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    r = fn(*args)
    for k in env:
        monkeypatch.delenv(k)
    return r


FUSED = {"MACM_TDM_SPLIT_OBS": "0", "MACM_TDM_TAIL_OBS": "0"}


@pytest.mark.parametrize("E,teams,kw,debug,K,workers", [
    (4096, [16, 16], {}, 0, 20, "steps=5"),                  # full chip: the last 5 steps in the tail
    (64, [16, 16], {}, 0, 33, "steps=3"),                    # the last 3 of 33 steps (balanced order)
    (512, [16, 16], {}, 0, 20, None),                        # C4's shard, observe-only blocks
    (512, [16, 16], {}, 0, 20, "0"),                         # the physics waves alone observe
    (4096, [16, 16], {}, 0, 20, None),                       # C4 on one GPU: every slot an env
    (37, [16, 16], {"obs_f64": True}, 0, 19, "3"),           # float64 obs (the pair tiles)
    (24, [32, 32], {}, 0, 9, None),                          # N = 64
    (64, [3, 3, 3], {"fresh_raycast": True}, 0, 33, None),   # >= 32 steps: the balanced env order
    (16, [8, 8], {"world_width": 8.0, "world_height": 8.0}, 0, 25, None),  # deaths
    (12, [16, 16], {}, _abi.DEBUG_FORCE_SPILL, 7, None),     # the spill step's snapshots
])
def test_tail_equals_fused(monkeypatch, E, teams, kw, debug, K, workers):
    """The tail observation (flock_step_w64.hip TailObs): each env's wave steps its K steps writing
    snapshots and publishing them; finished waves (and observe-only blocks) observe the (step, env)
    rows. Bit for bit the fused form's trajectory, state and counters, twice in a row (the second
    launch's tag and row counter)."""
    N = sum(teams)
    a, b = pair(monkeypatch, E, teams, 500 + E + N, debug, **kw)
    acts = actions(2 * K, E, N, 3 * E + N)
    env = {"MACM_TDM_SPLIT_OBS": "0", "MACM_TDM_TAIL_OBS": "1"}
    if workers is not None and workers.startswith("steps="):
        env["MACM_TDM_TAIL_STEPS"] = workers[6:]
    elif workers is not None:
        env["MACM_TDM_TAIL_WORKERS"] = workers
    for r in range(2):
        ta = call_env(monkeypatch, FUSED, a.rollout_traj, acts[r * K:(r + 1) * K])
        tb = call_env(monkeypatch, env, b.rollout_traj, acts[r * K:(r + 1) * K])
        for key in ta:
            assert torch.equal(ta[key], tb[key]), f"launch {r}: {key}"
        same_state(a, b, f"launch {r}")
    assert a.status() == 0 and b.status() == 0
    if debug:
        assert b.spilled() > 0


def test_reserve_then_rollouts(monkeypatch):
    """macm_tdm_reserve sizes the tail observation's snapshots ahead; rollouts shorter and longer than
    the reservation (the latter grows it) still equal the fused form."""
    E, teams = 64, [16, 16]
    a, b = pair(monkeypatch, E, teams, 31)
    b.reserve(40)
    acts = actions(70, E, 32, 8)
    for lo, hi in ((0, 5), (5, 45), (45, 70)):
        ta = call_env(monkeypatch, FUSED, a.rollout_traj, acts[lo:hi])
        tb = b.rollout_traj(acts[lo:hi])
        for key in ta:
            assert torch.equal(ta[key], tb[key]), f"steps {lo}..{hi}: {key}"
    same_state(a, b, "after the rollouts")
    assert b.launch_flags() & _abi.LAUNCH_TAIL_OBS
