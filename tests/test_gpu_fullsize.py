"""BASELINE configs at their full per-GPU sizes on the HIP path (M: 4096 x 64, C4: 4096 x 2x16,
C3: 4096 x 256 with 4 flocks, C5 shard: 2048 x 1024), checked through properties that do not
depend on the batch size:

1. every env is a function of its global env id (seeding) and its own actions only, so envs
   sampled across the full batch equal the CPU oracle run of that env ALONE: rewards,
   neighbour ids, collision flags and observations every step, the whole state (positions,
   velocities, angles, fat AABBs, sleep clocks, the ordered contact list with warm-start
   impulses) at the end, bit-exact (obs: float32 of the oracle's f64, <= 1 ulp);
2. invariants over every env of the batch: status 0, agent-step counter = E * N * K,
   neighbour ids in range and never the agent itself, rewards in {-1, 0, 1} with -1 exactly
   on the collided agents (binary mode), contact lists of valid, unique (a < b) pairs;
3. two runs of the full batch give identical states.
"""
import numpy as np
import pytest
import torch

from oracle import OracleTDM
from parity import assert_state_equal, f32_obs_mismatch, oracle_for
from test_gpu_tdm import assert_tdm_state_equal, random_actions

pytestmark = pytest.mark.gpu

from gym_macm.settings import flockSettings, to_config  # noqa: E402
from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402

SEED = 0x6D61636D


def env_slice(state, e, E):
    return {k: (v[e:e + 1] if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == E else v)
            for k, v in state.items()}


def sample_envs(E, rng, k=4):
    s = {0, 1, E // 2, E - 1}
    s.update(int(x) for x in rng.integers(0, E, size=k))
    return sorted(s)


def check_contact_lists(state, N):
    cnt = state["contact_count"]
    for e in range(cnt.shape[0]):
        ab = state["contact_ab"][e, :int(cnt[e])].astype(np.int64)
        a, b = ab & 0xFFFF, ab >> 16
        assert (a < b).all() and (b < N).all(), f"env {e}: invalid pair"
        assert len(np.unique(ab)) == len(ab), f"env {e}: duplicate pair"


def flock_full(E, N, steps, targets=None, max_contacts=None, n_sample=4, seed=SEED):
    kw = {} if max_contacts is None else dict(max_contacts=max_contacts)
    vec = FlockVec(E, n_agents=[N], targets=targets, seed=seed, device="cuda:0", **kw)
    cfg = to_config(flockSettings(), N, vec.n_targets, obs_f64=True)
    rng = np.random.default_rng(seed)
    envs = sample_envs(E, rng, n_sample)
    orcs = {e: oracle_for(cfg, vec.targets_idx, 1, seed, env_offset=e) for e in envs}
    vec.world.reset_counters()
    lane = np.arange(N)[None, :]
    for t in range(steps):
        a = rng.integers(0, 3, size=(E, N, 3)).astype(np.uint8)
        obs, nbr, rew, _ = vec.step(torch.from_numpy(a).cuda())
        nbr, rew = nbr.cpu().numpy(), rew.cpu().numpy()
        coll = vec.world.collided.cpu().numpy()
        obs = obs.cpu().numpy()
        # invariants over the whole batch
        assert ((nbr >= 0) & (nbr < N) & (nbr != lane)).all(), f"step {t}: neighbour id"
        assert np.isin(rew, (-1.0, 0.0, 1.0)).all(), f"step {t}: reward values"
        assert ((rew == -1.0) == (coll != 0)).all(), f"step {t}: -1 exactly on collided agents"
        # sampled envs against the oracle run of that env alone
        for e in envs:
            r = orcs[e].step(a[e:e + 1])
            np.testing.assert_array_equal(rew[e:e + 1], r["reward"].astype(np.float32), err_msg=f"rew env {e} step {t}")
            np.testing.assert_array_equal(nbr[e:e + 1], r["nbr_id"], err_msg=f"nbr env {e} step {t}")
            np.testing.assert_array_equal(coll[e:e + 1], r["collided"], err_msg=f"coll env {e} step {t}")
            f32_obs_mismatch(obs[e:e + 1], r["obs"])
    assert vec.status() == 0
    assert int(vec.counters()[0]) == E * N * steps
    s = vec.get_state()
    check_contact_lists(s, N)
    for e in envs:
        assert_state_equal(env_slice(s, e, E), orcs[e].get_state(vec.world.C), f"env {e}")
    return vec, s


def test_metric_config_full_size_4096x64():
    flock_full(4096, 64, 40)


def test_metric_config_full_size_deterministic():
    states = []
    for _ in range(2):
        vec = FlockVec(4096, n_agents=[64], seed=SEED, device="cuda:0")
        rng = np.random.default_rng(3)
        for _ in range(25):
            vec.step(torch.from_numpy(rng.integers(0, 3, size=(4096, 64, 3)).astype(np.uint8)).cuda())
        states.append(vec.get_state())
    assert_state_equal(states[0], states[1], "second full-size run")


def test_c3_full_size_4096x256_four_flocks():
    tg = [i // 64 for i in range(256)]
    flock_full(4096, 256, 40, targets=tg, max_contacts=4096, n_sample=2)


def test_c5_shard_full_size_2048x1024():
    flock_full(2048, 1024, 10, max_contacts=16384, n_sample=1)


def test_c4_tdm_full_size_4096x2x16():
    E, teams, steps = 4096, [16, 16], 40
    N = sum(teams)
    w = TdmWorld(tdm_config(teams), E, device="cuda:0")
    w.reset(SEED, 0)
    rng = np.random.default_rng(4)
    envs = sample_envs(E, rng)
    orcs = {e: OracleTDM(tdm_config(teams, obs_f64=True), 1, SEED, e) for e in envs}
    for t in range(steps):
        a = random_actions(rng, E, N)
        w.step(torch.from_numpy(a).cuda())
        health, alive, mask = w.health.cpu().numpy(), w.alive.cpu().numpy(), w.mask.cpu().numpy()
        obs = w.obs.cpu().numpy()
        # invariants: health only drops from 1 in steps of 0.25, dead agents are masked out
        assert ((health * 4 == np.round(health * 4)) & (health <= 1.0)).all(), f"step {t}: health values"
        assert (mask.sum(axis=2) <= (alive.sum(axis=1, keepdims=True) - alive)).all(), f"step {t}: mask"
        for e in envs:
            r = orcs[e].step(a[e:e + 1])
            np.testing.assert_array_equal(health[e:e + 1], r["health"], err_msg=f"health env {e} step {t}")
            np.testing.assert_array_equal(alive[e:e + 1], r["alive"], err_msg=f"alive env {e} step {t}")
            np.testing.assert_array_equal(mask[e:e + 1], r["mask"], err_msg=f"mask env {e} step {t}")
            f32_obs_mismatch(obs[e:e + 1], r["obs"])
    assert w.status() == 0
    s = w.get_state()
    check_contact_lists(s, N)
    for e in envs:
        assert_tdm_state_equal(env_slice(s, e, E), orcs[e].get_state(), f"env {e}")


# ---- the thinly sampled configs, at their own batch sizes and launch forms ------------

def sampled_oracles(cfg, tidx, envs, seed=SEED):
    return {e: oracle_for(cfg, tidx, 1, seed, env_offset=e) for e in envs}


def check_sampled_final(vec, orcs, last, E, ctx):
    """Final state and last outputs of the sampled envs equal their lone oracle runs."""
    s = vec.get_state()
    check_contact_lists(s, vec.N)
    obs, nbr, rew = vec.world.obs.cpu().numpy(), vec.world.nbr_id.cpu().numpy(), vec.world.reward.cpu().numpy()
    coll = vec.world.collided.cpu().numpy()
    for e, o in orcs.items():
        assert_state_equal(env_slice(s, e, E), o.get_state(vec.world.C), f"{ctx} env {e}")
        r = last[e]
        np.testing.assert_array_equal(rew[e:e + 1], r["reward"].astype(np.float32), err_msg=f"{ctx} rew env {e}")
        np.testing.assert_array_equal(nbr[e:e + 1], r["nbr_id"], err_msg=f"{ctx} nbr env {e}")
        np.testing.assert_array_equal(coll[e:e + 1], r["collided"], err_msg=f"{ctx} coll env {e}")
        f32_obs_mismatch(obs[e:e + 1], r["obs"])


def test_c5_shard_driver_launch_form_2048x1024():
    """The C5 shard as bench.py launches it: a W = 2 step rollout from reset, then a 30-step rollout
    (macm_world_rollout: kernel A, the dense envs' DFS kernel, the level solver and kernel C per
    step), against the lone oracle runs of 6 sampled envs over all 32 steps from reset."""
    E, N, W, K = 2048, 1024, 2, 30
    vec = FlockVec(E, n_agents=[N], seed=SEED, device="cuda:0")
    cfg = to_config(flockSettings(), N, 1, obs_f64=True)
    rng = np.random.default_rng(55)
    envs = sample_envs(E, rng, 2)
    assert len(envs) >= 4
    orcs = sampled_oracles(cfg, vec.targets_idx, envs)
    acts = torch.randint(0, 3, (W + K, E, N, 3), dtype=torch.uint8, device="cuda:0",
                         generator=torch.Generator(device="cuda:0").manual_seed(7))
    vec.world.rollout(acts[:W].contiguous())
    vec.world.reset_counters()
    vec.world.rollout(acts[W:].contiguous())
    a = acts.cpu().numpy()
    last = {}
    for e, o in orcs.items():
        for k in range(W + K):
            last[e] = o.step(a[k, e:e + 1])
    assert vec.status() == 0 and int(vec.counters()[0]) == E * N * K
    check_sampled_final(vec, orcs, last, E, "C5 driver form")


@pytest.mark.parametrize("launch", ["step", "rollout"])
def test_c2_full_size_1024x64(launch):
    """C2 (cm-flock-v0, 64 agents x 1024 envs) at its own batch size: below the scalar-sweep
    threshold, so the packed-sweep instantiations run (env_step_w64 / env_rollout_w64<0, 64,
    float, false>); 8 sampled envs against their lone oracle runs over 60 steps from reset."""
    E, N, K = 1024, 64, 60
    if launch == "step":
        flock_full(E, N, K, n_sample=4)
        return
    vec = FlockVec(E, n_agents=[N], seed=SEED, device="cuda:0")
    cfg = to_config(flockSettings(), N, 1, obs_f64=True)
    rng = np.random.default_rng(21)
    envs = sample_envs(E, rng, 4)
    orcs = sampled_oracles(cfg, vec.targets_idx, envs)
    a = rng.integers(0, 3, size=(K, E, N, 3)).astype(np.uint8)
    vec.world.rollout(torch.from_numpy(a).cuda())
    last = {e: None for e in envs}
    for e, o in orcs.items():
        for k in range(K):
            last[e] = o.step(a[k, e:e + 1])
    assert vec.status() == 0 and int(vec.counters()[0]) == E * N * K
    check_sampled_final(vec, orcs, last, E, "C2 rollout")


def test_c3_closed_loop_bots_full_size_4096x256():
    """C3 (256 agents, 4 flocks, 4096 envs) in the closed loop with the device bots.flock (the
    workgroup path, per-step launches and the bot kernel, in env slices) for 150 steps from reset:
    6 sampled envs against the oracle driven by the reference bot (test_scripts/bots.py:37-61) on
    its own observations rounded to the world's float32, final state and the bot's next actions."""
    from gym_macm.bots import flock_actions
    from parity import flock_bot
    E, N, K = 4096, 256, 150
    tg = [i // 64 for i in range(N)]
    vec = FlockVec(E, n_agents=[N], targets=tg, seed=SEED, device="cuda:0", max_contacts=4096)
    cfg = to_config(flockSettings(), N, vec.n_targets, obs_f64=True)
    rng = np.random.default_rng(31)
    envs = sample_envs(E, rng, 2)
    orcs = sampled_oracles(cfg, vec.targets_idx, envs)
    loop = flock_actions(vec.obs)
    vec.world.rollout_bots(loop, K)
    torch.cuda.synchronize()
    last = {}
    for e, o in orcs.items():
        obs, _ = o.observe()
        for k in range(K):
            last[e] = o.step(flock_bot(obs.astype(np.float32).astype(np.float64)))
            obs = last[e]["obs"]
    assert vec.status() == 0 and int(vec.counters()[0]) == E * N * K
    check_sampled_final(vec, orcs, last, E, "C3 closed loop")
    nxt = loop.cpu().numpy()
    for e in envs:
        np.testing.assert_array_equal(nxt[e:e + 1], flock_bot(last[e]["obs"].astype(np.float32).astype(np.float64)),
                                      err_msg=f"the bot's next actions, env {e}")
