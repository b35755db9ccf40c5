"""HIP path vs the CPU oracle, through the C-ABI (libmacm_hip.so).

Bar: bit-exact for positions, velocities, angles, fat AABBs, sleep clocks, the
ordered contact list with warm-start impulses, neighbour ids, rewards and done, and the
reward sums (per env and in total, in the device's fixed float64 order) of every rollout;
observations (float32) equal the oracle's f64 values rounded to f32, with at most
1 ulp allowed where double atan2/sin/cos of ocml and glibc round differently."""
import numpy as np
import pytest
import torch

import goldens
from parity import assert_state_equal, f32_obs_mismatch, oracle_for

pytestmark = pytest.mark.gpu

from gym_macm.dist import env_order_sum, pairwise_reward_sum  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402


def make_pair(E, n_agents, seed, targets=None, env_offset=0, obs_dtype=torch.float32, **kw):
    vec = FlockVec(E, n_agents=n_agents, targets=targets, seed=seed, env_offset=env_offset,
                   device="cuda:0", obs_dtype=obs_dtype, **kw)
    N = vec.N
    cfg = to_config(flockSettings(**kw), N, vec.n_targets, obs_f64=True)
    orc = oracle_for(cfg, vec.targets_idx, E, seed, env_offset)
    return vec, orc


def rand_actions(rng, E, N):
    return rng.integers(0, 3, size=(E, N, 3)).astype(np.uint8)


def obs_check(gpu_obs, oracle_obs64, obs_f64, ctx):
    """f32 obs: the oracle's f64 values rounded to f32 (<= 1 ulp, see parity.py);
    f64 obs: within a few f64 ulp (goldens.obs_close)."""
    if not obs_f64:
        return f32_obs_mismatch(gpu_obs, oracle_obs64)
    od = gpu_obs.shape[-1]
    for e in range(gpu_obs.shape[0]):
        assert goldens.obs_close(gpu_obs[e], oracle_obs64[e], od), f"obs {ctx} env {e}"
    return 0


def check_rollout(vec, orc, steps, rng, state_every=1, actions_fn=None, obs_f64=False):
    E, N = vec.num_envs, vec.N
    C = vec.world.C
    assert_state_equal(vec.get_state(), orc.get_state(C), "reset")
    vec.observe()
    o0, n0 = orc.observe()
    np.testing.assert_array_equal(vec.nbr_id.cpu().numpy(), n0)
    obs_check(vec.obs.cpu().numpy(), o0, obs_f64, "reset")
    ulp_total = 0
    vec.world.reset_counters()
    rs = np.zeros(E, np.float64)  # the reward sums in the device's order (macm_world_reward_sums)
    for t in range(steps):
        a = actions_fn(t) if actions_fn else rand_actions(rng, E, N)
        obs, nbr, rew, done = vec.step(torch.from_numpy(a).cuda())
        r = orc.step(a)
        rs += pairwise_reward_sum(r["reward"])
        np.testing.assert_array_equal(rew.cpu().numpy(), r["reward"].astype(np.float32), err_msg=f"reward step {t}")
        np.testing.assert_array_equal(nbr.cpu().numpy(), r["nbr_id"], err_msg=f"nbr step {t}")
        np.testing.assert_array_equal(done.cpu().numpy(), r["done"], err_msg=f"done step {t}")
        np.testing.assert_array_equal(vec.world.collided.cpu().numpy(), r["collided"], err_msg=f"coll step {t}")
        ulp_total += obs_check(obs.cpu().numpy(), r["obs"], obs_f64, f"step {t}")
        if (t + 1) % state_every == 0 or t == steps - 1:
            assert_state_equal(vec.get_state(), orc.get_state(C), f"step {t}")
    assert vec.status() == 0
    per_env, total = vec.reward_sums()
    np.testing.assert_array_equal(per_env, rs, err_msg="per-env reward sums")
    assert total == env_order_sum(rs), "reward total"
    return ulp_total


def test_reset_matches_reference_rng():
    vec, orc = make_pair(8, [64], seed=1234)
    assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), "reset")


def test_metric_config_rollout_bit_exact():
    vec, orc = make_pair(32, [64], seed=7)
    check_rollout(vec, orc, 150, np.random.default_rng(0), state_every=10)


def test_dense_start_multibody_islands():
    # start_spread 6: 64 agents in 36 m^2 -> heavy overlap, large islands, long DFS
    vec, orc = make_pair(16, [64], seed=3, start_spread=6)
    check_rollout(vec, orc, 120, np.random.default_rng(1), state_every=5)


def test_noop_actions_reach_sleep():
    # NOOP forces: bodies decelerate and fall asleep (v := 0) after 0.5 s below 0.01 m/s
    vec, orc = make_pair(8, [16], seed=5, start_spread=8)
    E, N = 8, 16
    noop = np.ones((E, N, 3), np.uint8)
    check_rollout(vec, orc, 160, None, state_every=20, actions_fn=lambda t: noop)
    s = vec.get_state()
    assert (s["vel"] == 0).all()


def test_small_configs_and_settings():
    for kw in (dict(n_agents=[4], seed=0), dict(n_agents=[5, 7], seed=21, targets=[0, 1, 2] * 4),
               dict(n_agents=[16], seed=3, targets=[0] * 8 + [1] * 8, reward_mode="linear", coord="cartesian"),
               dict(n_agents=[6], seed=2, hz=30.0, time_limit=1.0),
               dict(n_agents=[33], seed=9, velocityIterations=3, positionIterations=1)):
        kw = dict(kw)
        n_agents = kw.pop("n_agents")
        seed = kw.pop("seed")
        vec, orc = make_pair(6, n_agents, seed, **kw)
        check_rollout(vec, orc, 60, np.random.default_rng(seed), state_every=15)


def test_continuous_actions():
    vec, orc = make_pair(8, [12], seed=4, action_mode="continuous")
    rng = np.random.default_rng(4)
    E, N = 8, 12

    def acts(t):
        return rng.uniform(-1, 1, size=(E, N, 2)).astype(np.float32)

    C = vec.world.C
    for t in range(80):
        a = acts(t)
        _, nbr, rew, _ = vec.step(torch.from_numpy(a).cuda())
        r = orc.step(a)
        np.testing.assert_array_equal(rew.cpu().numpy(), r["reward"].astype(np.float32))
        np.testing.assert_array_equal(nbr.cpu().numpy(), r["nbr_id"])
    assert_state_equal(vec.get_state(), orc.get_state(C), "continuous")


def test_state_injection_from_oracle():
    """Inject an oracle state reached after 40 steps into a fresh GPU world."""
    E, N = 8, 64
    vec, orc = make_pair(E, [N], seed=11, start_spread=10)
    rng = np.random.default_rng(2)
    for _ in range(40):
        orc.step(rand_actions(rng, E, N))
    vec.set_state(orc.get_state(vec.world.C))
    check_rollout(vec, orc, 40, rng, state_every=10)


def test_shard_offsets_are_slices_of_the_full_batch():
    full = FlockVec(8, n_agents=[64], seed=99, device="cuda:0")
    part = FlockVec(4, n_agents=[64], seed=99, env_offset=4, device="cuda:0")
    rng = np.random.default_rng(5)
    for _ in range(30):
        a = rand_actions(rng, 8, 64)
        _, _, rf, _ = full.step(torch.from_numpy(a).cuda())
        _, _, rp, _ = part.step(torch.from_numpy(a[4:]).cuda())
        np.testing.assert_array_equal(rf.cpu().numpy()[4:], rp.cpu().numpy())
    sf, sp = full.get_state(), part.get_state()
    np.testing.assert_array_equal(sf["pos"][4:], sp["pos"])


def test_determinism_two_runs_identical():
    rng = np.random.default_rng(8)
    acts = [rand_actions(rng, 16, 64) for _ in range(40)]
    outs = []
    for _ in range(2):
        v = FlockVec(16, n_agents=[64], seed=5, device="cuda:0")
        for a in acts:
            v.step(torch.from_numpy(a).cuda())
        outs.append(v.get_state())
    assert_state_equal(outs[0], outs[1], "second run")


def test_counters():
    v = FlockVec(8, n_agents=[32], seed=1, device="cuda:0")
    v.world.reset_counters()
    a = torch.ones((8, 32, 3), dtype=torch.uint8, device="cuda:0")
    coll = 0
    for _ in range(5):
        v.step(a)
        coll += int(v.world.collided.sum().item())
    c = v.counters()
    assert c[0] == 5 * 8 * 32 and c[1] == coll


@pytest.mark.parametrize("name", goldens.names())
def test_dropin_flock_matches_reference_goldens(name):
    """The drop-in dict API (gym_macm.envs.Flock over the HIP world) reproduces the
    reference env's own outputs (tests/golden, made from mvmnt.py)."""
    import random
    from gym_macm.envs import Flock
    g = goldens.load(name)
    m = g["meta"]
    random.seed(m["seed"])
    env = Flock(n_agents=m["n_agents"], targets=m["targets"], device="cuda:0", **m["kwargs"])
    N = m["N"]
    for t in range(m["steps"]):
        if m["policy"] == "random_cont":
            acts = {i: g["actions"][t][i].astype(np.float32) for i in range(N)}
        else:
            acts = {i: g["actions"][t][i].astype(np.int64) for i in range(N)}
        obs, rewards = env.step(acts)
        assert [rewards[i] for i in range(N)] == list(g["reward"][t]), f"rewards step {t}"
        # the reference's insertion order (contact agents first, world.contacts order)
        assert list(rewards.keys()) == [int(x) for x in g["reward_order"][t]], f"reward dict order step {t}"
        nbr = np.array([obs[i]["nodes"][0]["id"] for i in range(N)])
        np.testing.assert_array_equal(nbr, g["nbr"][t], err_msg=f"nbr step {t}")
        pos = np.array([np.concatenate([obs[i]["nodes"][0]["position"], obs[i]["nodes"][1]["position"]])
                        for i in range(N)])
        assert goldens.obs_close(pos, g["obs"][t], pos.shape[1]), f"obs step {t}"
        assert env.done == bool(g["done"][t])
    s = env.world.get_state()
    np.testing.assert_array_equal(s["pos"][0], g["pos"][-1])
    np.testing.assert_array_equal(s["angle"][0], g["angle"][-1])


# ---- workgroup-per-env kernel (64 < N <= 1024) ---------------------------------------


@pytest.mark.parametrize("n", [65, 100, 128])
def test_workgroup_kernel_sizes(n):
    vec, orc = make_pair(6, [n], seed=n, start_spread=12)
    check_rollout(vec, orc, 50, np.random.default_rng(n), state_every=10)


def test_c3_multiflock_256_agents_4_targets():
    """BASELINE config 3: n_agents=256, targets = i // 64 (4 flocks, README.md:44)."""
    tg = [i // 64 for i in range(256)]
    vec, orc = make_pair(4, [256], seed=33, targets=tg)
    assert vec.n_targets == 4
    check_rollout(vec, orc, 40, np.random.default_rng(3), state_every=10)


def test_c5_dense_1024_agents():
    """BASELINE config 5 shape: 1024 agents in the default 20 m spread (804 m^2 of
    circles in 400 m^2): one giant island, thousands of touching contacts."""
    vec, orc = make_pair(2, [1024], seed=55)
    check_rollout(vec, orc, 6, np.random.default_rng(5), state_every=2)


@pytest.mark.parametrize("vel,pos,warm", [(8, 3, True), (3, 1, True), (1, 0, False), (10, 2, False)])
def test_dense_relaxing_big_islands(vel, pos, warm):
    """Dense start that relaxes: islands of hundreds of contacts (the solver's chunked
    whole-wave path) whose position passes stop early once separated, with the solver
    settings varied (iterations, no position passes, no warm start)."""
    kw = dict(start_spread=11, velocityIterations=vel, positionIterations=pos, enableWarmStarting=warm)
    vec, orc = make_pair(3, [300], seed=300 + vel, **kw)
    check_rollout(vec, orc, 60, np.random.default_rng(vel), state_every=10)


def test_relaxed_lattice_big_island_early_exit():
    """A 256-body hexagonal cluster at spacing 0.995 (every neighbour pair touching, overlap
    0.005 < 3 * linearSlop): one island of ~700 contacts whose position passes stop after the
    first pass, inside the solver's chunked whole-wave path. The state is injected into both
    the oracle and the HIP world."""
    E, N = 2, 256
    vec, orc = make_pair(E, [N], seed=7)
    C = vec.world.C
    st = orc.get_state(C)
    s, h = 0.995, 0.995 * np.sqrt(3.0) / 2.0
    k, i = np.divmod(np.arange(N), 16)
    pos = np.stack([(i + 0.5 * (k % 2)) * s - 8.0, k * h - 7.0], -1).astype(np.float32)
    for e in range(E):
        p = pos + np.float32(0.3 * e)
        st["pos"][e] = p
        st["vel"][e] = 0.0
        st["sleep"][e] = 0.0
        r = np.float32(0.5 + 0.1)
        st["fat"][e] = np.concatenate([p - r, p + r], -1)
        f = st["fat"][e]
        pairs = [(a, b) for a in range(N - 1, -1, -1) for b in range(N - 1, a, -1)
                 if not (f[b, 0] > f[a, 2] or f[b, 1] > f[a, 3] or f[a, 0] > f[b, 2] or f[a, 1] > f[b, 3])]
        assert len(pairs) <= C
        st["contact_count"][e] = len(pairs)
        st["contact_ab"][e] = 0
        st["contact_ab"][e, :len(pairs)] = [a | (b << 16) for a, b in pairs]
        st["contact_imp"][e] = 0.0
    orc.set_state(st)
    vec.set_state(st)
    rng = np.random.default_rng(17)
    check_rollout(vec, orc, 30, rng, state_every=5,
                  actions_fn=lambda t: np.ones((E, N, 3), np.uint8) if t < 5 else rand_actions(rng, E, N))
