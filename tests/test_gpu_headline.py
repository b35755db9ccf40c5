"""The benchmark's exact launches against the CPU oracle, over EVERY env of the metric config.

bench.py (the driver runs `--steps 20 --warmup 5`) times one `macm_world_rollout` launch of K = 20
steps over 4096 envs x 64 agents after a W = 5-step rollout from reset (seed 0x6d61636d, actions
drawn on the device by torch.randint from seed + 1). At >= 2048 envs that launch is the
scalar-sweep instantiation `env_rollout_w64<0, 64, float, true>`, which the smaller rollout tests
never reach. Here the same launches run with the same actions, and the oracle (oracle/, the C
restatement of gym_macm/envs/mvmnt.py:81-140 over b2lite) steps all 4096 envs with them:

  * the whole state of every env after the K steps (positions, velocities, angles, fat AABBs,
    sleep clocks, the ordered contact list with its warm-start impulses, step count, time) bit-exact;
  * the last step's rewards, neighbour ids, collision flags (bit-exact) and observations (float32 of
    the oracle's float64, <= 1 ulp) of every agent;
  * the world's counters over the K timed steps = the oracle's per-step outputs summed over them,
    and the reward sums (per env and in total, float64) = the oracle's rewards summed in the
    device's fixed order (gym_macm.dist.pairwise_reward_sum), bit for bit.

The closed loop (`--policy bots`, macm_world_rollout_bots with the device bots.flock) is pinned the
same way, the oracle driven by the reference's bot (tests/parity.py flock_bot) on its own
observations rounded to float32, which is what the device bot sees."""
import numpy as np
import pytest
import torch

from parity import assert_state_equal, f32_obs_mismatch, flock_bot, oracle_for

pytestmark = pytest.mark.gpu

from gym_macm.bots import flock_actions  # noqa: E402
from gym_macm.dist import env_order_sum, pairwise_reward_sum  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402

SEED = 0x6D61636D
E, N, W, K = 4096, 64, 5, 20
THREADS = 16


def oracle():
    return oracle_for(to_config(flockSettings(), N, 1, obs_f64=True), None, E, SEED)


def check_last_outputs(vec, r):
    np.testing.assert_array_equal(vec.world.reward.cpu().numpy(), r["reward"].astype(np.float32))
    np.testing.assert_array_equal(vec.nbr_id.cpu().numpy(), r["nbr_id"])
    np.testing.assert_array_equal(vec.world.collided.cpu().numpy(), r["collided"])
    np.testing.assert_array_equal(vec.world.done.cpu().numpy(), r["done"])
    f32_obs_mismatch(vec.obs.cpu().numpy(), r["obs"])


def check_reward_sums(vec, rs):
    per_env, total = vec.reward_sums()
    np.testing.assert_array_equal(per_env, rs, err_msg="per-env reward sums")
    assert total == env_order_sum(rs)


def test_headline_rollout_launch_all_envs_match_oracle():
    vec = FlockVec(E, n_agents=[N], seed=SEED, device="cuda:0")
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(SEED + 1)  # bench.py, rank 0
    acts = torch.randint(0, 3, (W + K, E, N, 3), dtype=torch.uint8, device="cuda:0", generator=gen)
    vec.world.rollout_raw(acts.data_ptr(), W, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    vec.world.reset_counters()
    vec.world.rollout_raw(acts[W:].data_ptr(), K, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    a = acts.cpu().numpy()
    orc = oracle()
    tot = np.zeros(4, np.int64)
    rs = np.zeros(E, np.float64)
    for k in range(W + K):
        r = orc.step(a[k], n_threads=THREADS)
        if k >= W:
            tot += [E * N, int(r["collided"].sum()), int((r["reward"] > 0).sum()), int(r["done"].sum())]
            rs += pairwise_reward_sum(r["reward"])
    assert vec.status() == 0
    assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), "after the timed launch")
    check_last_outputs(vec, r)
    np.testing.assert_array_equal(vec.counters(), tot)
    check_reward_sums(vec, rs)
    assert tot[1] > 0


def test_headline_trajectory_launch_all_envs_match_oracle():
    """The driver's exact timed launch (bench.py's default `--outputs trajectory`: one
    macm_world_rollout_traj of K = 20 steps after the W = 5-step warm-up rollout), pinned row by row:
    trajectory row k (rewards, neighbour ids, collision flags, done bit-exact; observations <= 1 ulp of
    the oracle's float64 rounded to float32) equals the oracle's step W + k over all 4096 envs, and the
    state after the launch, the counters and the reward sums equal the oracle's."""
    vec = FlockVec(E, n_agents=[N], seed=SEED, device="cuda:0")
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(SEED + 1)  # bench.py, rank 0
    acts = torch.randint(0, 3, (W + K, E, N, 3), dtype=torch.uint8, device="cuda:0", generator=gen)
    sh = torch.cuda.current_stream().cuda_stream
    traj = vec.world.trajectory_buffers(K)
    vec.world.rollout_raw(acts.data_ptr(), W, sh)
    torch.cuda.synchronize()
    vec.world.reset_counters()
    vec.world.rollout_traj_raw(acts[W:].data_ptr(), K, traj, sh)  # bench.py's timed call
    torch.cuda.synchronize()
    a = acts.cpu().numpy()
    rows = {k: v.cpu().numpy() for k, v in traj.items()}
    orc = oracle()
    tot = np.zeros(4, np.int64)
    rs = np.zeros(E, np.float64)
    for k in range(W + K):
        r = orc.step(a[k], n_threads=THREADS)
        if k < W:
            continue
        j = k - W
        np.testing.assert_array_equal(rows["reward"][j], r["reward"].astype(np.float32), err_msg=f"reward row {j}")
        np.testing.assert_array_equal(rows["nbr_id"][j], r["nbr_id"], err_msg=f"nbr_id row {j}")
        np.testing.assert_array_equal(rows["collided"][j], r["collided"], err_msg=f"collided row {j}")
        np.testing.assert_array_equal(rows["done"][j], r["done"], err_msg=f"done row {j}")
        f32_obs_mismatch(rows["obs"][j], r["obs"])
        tot += [E * N, int(r["collided"].sum()), int((r["reward"] > 0).sum()), int(r["done"].sum())]
        rs += pairwise_reward_sum(r["reward"])
    assert vec.status() == 0
    assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), "after the trajectory launch")
    np.testing.assert_array_equal(vec.counters(), tot)
    check_reward_sums(vec, rs)
    assert tot[1] > 0


def test_headline_closed_loop_launch_all_envs_match_oracle():
    vec = FlockVec(E, n_agents=[N], seed=SEED, device="cuda:0")
    loop = flock_actions(vec.obs)
    sh = torch.cuda.current_stream().cuda_stream
    vec.world.rollout_bots_raw(loop.data_ptr(), W, sh)
    torch.cuda.synchronize()
    vec.world.reset_counters()
    vec.world.rollout_bots_raw(loop.data_ptr(), K, sh)
    torch.cuda.synchronize()
    orc = oracle()
    obs, _ = orc.observe()
    tot = np.zeros(4, np.int64)
    rs = np.zeros(E, np.float64)
    for k in range(W + K):
        act = flock_bot(obs.astype(np.float32).astype(np.float64))
        r = orc.step(act, n_threads=THREADS)
        obs = r["obs"]
        if k >= W:
            tot += [E * N, int(r["collided"].sum()), int((r["reward"] > 0).sum()), int(r["done"].sum())]
            rs += pairwise_reward_sum(r["reward"])
    assert vec.status() == 0
    assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), "after the closed-loop launch")
    check_last_outputs(vec, r)
    np.testing.assert_array_equal(vec.counters(), tot)
    check_reward_sums(vec, rs)
    np.testing.assert_array_equal(loop.cpu().numpy(), flock_bot(obs.astype(np.float32).astype(np.float64)),
                                  err_msg="the bot's next actions")
