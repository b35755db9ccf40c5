"""TDM with more than 64 agents per env: the workgroup TDM step (csrc/tdm_step_wg.hip).

The reference's TDM takes any team sizes (combat.py:82-83) in an uncapped b2World
(cm_framework.py:161). The wave kernel holds one agent per lane (N <= 64); above that every env is
stepped by one workgroup: the action loop with the melee ray casts and the shared listener
(combat.py:121-155), deaths (:157-165), then the spill step's physics (HBM working set) and TDM's
observation / done / winner (:166-182, 206-227). Bar: every state field, the health / alive / done
/ winner / mask outputs and the observation equal the oracle's (oracle/tdm_oracle.c over b2lite)
at every step, status 0; the rollout forms equal the per-step launches."""
import numpy as np
import pytest
import torch

from oracle import OracleTDM
from parity import combat_bot
from test_gpu_tdm import assert_tdm_state_equal, check_obs, check_rollout, make_pair, random_actions

pytestmark = pytest.mark.gpu

from gym_macm import _abi  # noqa: E402
from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402


@pytest.mark.parametrize("teams,kw,policy,steps", [
    ([40, 40], dict(world_width=16.0, world_height=16.0), "bot", 150),     # 80: two waves
    ([33, 32], {}, "random", 60),                                          # 65: one body past a wave
    ([30, 30, 30, 30], dict(obs_f64=True, world_width=20.0, world_height=20.0), "bot", 120),
    ([50, 50], dict(fresh_raycast=True, decay_mov_penalty=True, world_width=14.0, world_height=14.0), "bot", 120),
    ([100, 100], dict(world_width=12.0, world_height=12.0), "random", 40),  # crowded: big islands
])
def test_tdm_wg_matches_oracle(teams, kw, policy, steps):
    E, N = 4, sum(teams)
    w, orc = make_pair(E, teams, seed=N + 11, **kw)
    rng = np.random.default_rng(N)
    pol = combat_bot if policy == "bot" else (lambda o, m: random_actions(rng, E, N, p_attack=0.4))
    r = check_rollout(w, orc, steps, pol, state_every=10)
    assert int(w.counters()[1]) > 0, "no melee attack"
    assert w.spilled() == steps * E, "every env-step above 64 agents is the workgroup step's"
    if policy == "bot":
        assert (r["alive"] == 0).any(), "no death: the deaths / inactive-body path was not exercised"


def test_tdm_wg_large_teams():
    """2 x 256 agents (512 per env, eight waves per workgroup) for 25 steps from the crowded
    30 x 30 spawn, and 2 x 512 (the 1024-agent cap) for 5."""
    for teams, steps in (([256, 256], 25), ([512, 512], 5)):
        E, N = 2, sum(teams)
        w, orc = make_pair(E, teams, seed=N)
        rng = np.random.default_rng(N)
        check_rollout(w, orc, steps, lambda o, m: random_actions(rng, E, N, p_attack=0.5), state_every=5)


def test_tdm_wg_cap_and_refusal():
    # up to 4096 agents since round 5 (tests/test_gpu_big.py); one more is refused
    with pytest.raises(_abi.MacmError):
        TdmWorld(tdm_config([2049, 2048]), 1, device="cuda:0")


@pytest.mark.parametrize("bots", [False, True])
def test_tdm_wg_rollouts_equal_per_step(bots):
    """macm_tdm_rollout(_bots) and the trajectory forms on the workgroup path (one launch per step,
    and the bots kernel's) equal K step() calls: outputs, every step's trajectory row, state,
    counters and, in the closed loop, the bot's actions."""
    from gym_macm.bots import combat_actions
    E, teams, K = 8, [48, 40], 30
    N = sum(teams)
    cfg = dict(world_width=14.0, world_height=14.0)
    a = TdmWorld(tdm_config(teams, **cfg), E, device="cuda:0")
    b = TdmWorld(tdm_config(teams, **cfg), E, device="cuda:0")
    c = TdmWorld(tdm_config(teams, **cfg), E, device="cuda:0")
    for x in (a, b, c):
        x.reset(5, 0)
    rows = []
    if bots:
        act_a = combat_actions(a.obs, a.mask)
        act_b = act_a.clone()
        act_c = torch.empty((K + 1, E, N, 4), dtype=torch.uint8, device="cuda:0")
        act_c[0] = act_a
        for _ in range(K):
            a.step(act_a)
            rows.append([t.clone() for t in a.outputs()])
            combat_actions(a.obs, a.mask, out=act_a)
        b.rollout_bots(act_b, K)
        traj = c.rollout_bots_traj(act_c, K)
        assert torch.equal(act_a, act_b) and torch.equal(act_c[K], act_a), "the bot's next actions"
    else:
        g = torch.Generator(device="cuda:0")
        g.manual_seed(2)
        acts = torch.randint(0, 3, (K, E, N, 4), dtype=torch.uint8, device="cuda:0", generator=g)
        acts[..., 3] = torch.randint(0, 2, (K, E, N), dtype=torch.uint8, device="cuda:0", generator=g)
        for k in range(K):
            a.step(acts[k])
            rows.append([t.clone() for t in a.outputs()])
        b.rollout(acts)
        traj = c.rollout_traj(acts)
    for x, y in zip(a.outputs(), b.outputs()):
        assert torch.equal(x, y)
    keys = TdmWorld._TRAJ_KEYS
    for k in range(K):
        out_k = dict(zip(keys, rows[k]))
        for key in keys:
            assert torch.equal(traj[key][k], out_k[key]), f"trajectory row {k} {key}"
    for x in (b, c):
        sa, sx = a.get_state(), x.get_state()
        for key in sa:
            np.testing.assert_array_equal(sa[key], sx[key], err_msg=f"state[{key}]")
        np.testing.assert_array_equal(a.counters(), x.counters())
    assert int(a.counters()[1]) > 0


def test_tdm_wg_reset_envs_and_autoreset_on_done():
    """Per-env resets (macm_tdm_reset_envs: poses from each env's MT19937 stream, the init kernel
    of the workgroup path) against the oracle's reset_envs, over episodes that end by a wipe-out."""
    E, teams = 6, [40, 30]
    cfg = dict(world_width=10.0, world_height=10.0)
    w = TdmWorld(tdm_config(teams, **cfg), E, device="cuda:0")
    w.reset(41)
    orc = OracleTDM(tdm_config(teams, obs_f64=True, **cfg), E, 41)
    obs, mask = orc.observe()
    resets = 0
    for t in range(400):
        a = combat_bot(obs, mask)
        w.step(torch.from_numpy(a).cuda())
        r = orc.step(a)
        if r["done"].any():
            w.reset_envs(w.done)
            orc.reset_envs(r["done"])
            resets += int(r["done"].sum())
        obs, mask = orc.observe()
        if t % 25 == 24:
            assert_tdm_state_equal(w.get_state(), orc.get_state(), f"step {t}")
    assert_tdm_state_equal(w.get_state(), orc.get_state(), "end")
    np.testing.assert_array_equal(w.mask.cpu().numpy(), mask)
    w.observe()
    check_obs(w, obs, mask, "observe after resets")
    assert resets > 0, "no episode ended"


def test_tdm_wg_state_injection():
    """set_state of an oracle state mid-episode (dead bodies, a primed listener) continues
    identically on the workgroup path."""
    E, teams = 3, [36, 36]
    w, orc = make_pair(E, teams, seed=8, world_width=12.0, world_height=12.0)
    obs, mask = orc.observe()
    for _ in range(60):
        r = orc.step(combat_bot(obs, mask))
        obs, mask = r["obs"], r["mask"]
    assert (r["alive"] == 0).any()
    w.set_state(orc.get_state())
    w.observe()
    np.testing.assert_array_equal(w.mask.cpu().numpy(), mask)
    check_rollout(w, orc, 40, combat_bot, state_every=10)


def test_tdm_wg_dict_api():
    """The drop-in TDM (gym_macm.envs.TDM, the reference's dict API) with 2 x 40 agents: steps
    through the workgroup path, every alive agent sees every other alive agent."""
    from gym_macm.envs import TDM
    env = TDM(n_agents=[40, 40])
    assert len(env.agents) == 80
    ids = [a.id for a in env.agents]
    assert ids[0] == "00" and ids[40] == "10"
    rng = np.random.default_rng(0)
    for _ in range(20):
        acts = {aid: np.array([rng.integers(3), rng.integers(3), rng.integers(3), rng.integers(2)])
                for aid in env.obs}
        obs = env.step(acts)
        for aid, o in obs.items():
            assert len(o["agents"]) == len(obs) - 1


def test_lds_limits_only_grow():
    """The workgroup kernels' dynamic-LDS limits are per kernel, not per world: creating a smaller
    world after a larger one must not make the larger world's launches (88 KB at 1024 agents,
    above the default 64 KB) fail. TDM and Flock."""
    from gym_macm.vec import FlockVec
    big = TdmWorld(tdm_config([512, 512]), 1, device="cuda:0")
    big.reset(1)
    small = TdmWorld(tdm_config([40, 40]), 1, device="cuda:0")
    small.reset(2)
    rng = np.random.default_rng(0)
    big.step(torch.from_numpy(random_actions(rng, 1, 1024)).cuda())
    small.step(torch.from_numpy(random_actions(rng, 1, 80)).cuda())
    torch.cuda.synchronize()
    assert big.status() == 0 and small.status() == 0
    fbig = FlockVec(2, n_agents=[1024], seed=3, device="cuda:0")
    fsmall = FlockVec(2, n_agents=[100], seed=4, device="cuda:0")
    fbig.step(torch.ones((2, 1024, 3), dtype=torch.uint8, device="cuda:0"))
    fsmall.step(torch.ones((2, 100, 3), dtype=torch.uint8, device="cuda:0"))
    torch.cuda.synchronize()
    assert fbig.status() == 0 and fsmall.status() == 0


def test_tdm_wg_pooled_slots_match_one_slot_per_env():
    """above 64 agents every TDM env-step takes the spill step, so a pooled working set
    (fewer slots than envs) is on the main path. The workgroup step takes its slot before it commits
    anything and returns it before the O(N^2) observation. 12 envs sharing 3 slots (and then 1) over
    several steps equal the world with a slot per env, bit for bit, status 0; clearing the flag brings
    back the world's own slots."""
    E, teams, K = 12, [40, 40], 12
    N = sum(teams)
    kw = dict(world_width=14.0, world_height=14.0)
    a = TdmWorld(tdm_config(teams, **kw), E, device="cuda:0")
    b = TdmWorld(tdm_config(teams, **kw), E, device="cuda:0")
    for x in (a, b):
        x.reset(17, 0)
    rng = np.random.default_rng(3)
    for k in range(K):
        b.set_debug(_abi.DEBUG_SPILL_POOL | ((3 if k < K // 2 else 1) << 8))
        acts = torch.from_numpy(random_actions(rng, E, N, p_attack=0.5)).cuda()
        a.step(acts)
        b.step(acts)
        for x, y in zip(a.outputs(), b.outputs()):
            assert torch.equal(x, y), f"step {k}"
    b.set_debug(0)
    assert b.status() == 0 and a.status() == 0
    sa, sb = a.get_state(), b.get_state()
    for key in sa:
        np.testing.assert_array_equal(sa[key], sb[key], err_msg=f"state[{key}]")
    np.testing.assert_array_equal(a.counters(), b.counters())
    with pytest.raises(_abi.MacmError):  # more slots than allocated
        b.set_debug(_abi.DEBUG_SPILL_POOL | ((E + 1) << 8))


def test_tdm_wg_state_moves_only_the_used_lists():
    """get_state's contact rows hold max(contact_count) entries (ABI 7 contact_stride),
    not C = N(N-1)/2 (523,776 at 1024 agents), and set_state takes such rows back."""
    E, teams = 2, [512, 512]
    w, orc = make_pair(E, teams, seed=5)
    rng = np.random.default_rng(5)
    for _ in range(3):
        w.step(torch.from_numpy(random_actions(rng, E, 1024)).cuda())
    st = w.get_state()
    n = int(st["contact_count"].max())
    assert 0 < n < w.C // 10 and st["contact_ab"].shape == (E, n) and st["contact_imp"].shape == (E, n, 2)
    twin = TdmWorld(tdm_config(teams), E, device="cuda:0")
    twin.reset(99, 0)
    twin.set_state(st)
    acts = torch.from_numpy(random_actions(rng, E, 1024)).cuda()
    w.step(acts)
    twin.step(acts)
    s1, s2 = w.get_state(), twin.get_state()
    for key in s1:
        np.testing.assert_array_equal(s1[key], s2[key], err_msg=f"state[{key}]")
