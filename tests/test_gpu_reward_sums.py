"""The reward sum (Σ of get_rewards' values, mvmnt.py:160-179) on the device.

macm_world_reward_sums keeps one float64 total per env: each step's float32 rewards summed pairwise
over the agent slots (flock_common.hpp block_pairwise_sum), added in step order. The host
restatement is gym_macm.dist.pairwise_reward_sum; the total over envs is their sum in env order
(gym_macm.dist.env_order_sum), which the multi-GPU path reproduces at any rank count
(tests/test_distributed.py). Bar: bit-exact against the oracle's rewards (binary mode is an integer
count, so the linear mode — values like 1 - d/35 — is what tests the order) in every launch form
and step path: the wave kernel per step and in one rollout launch, the workgroup path with a
number of waves that is not a power of two, the env slices on their own streams, the spill step,
the trajectory form at the metric size (self-consistency with the rewards it returns) and the
closed loop. Every tests/ rollout through test_gpu_parity.check_rollout checks the sums too, in
binary mode as well, where the library reads an env's total from its counters (positive-reward minus
collided agent-steps: the same bits, every partial sum of -1 / 0 / +1 values being an exact integer)
instead of accumulating it in the kernels."""
import numpy as np
import pytest
import torch

from test_gpu_parity import check_rollout, make_pair, rand_actions

pytestmark = pytest.mark.gpu

from gym_macm import _abi  # noqa: E402
from gym_macm.dist import env_order_sum, pairwise_reward_sum  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402


def assert_sums(vec, rs, ctx):
    per_env, total = vec.reward_sums()
    np.testing.assert_array_equal(per_env, rs, err_msg=f"{ctx}: per-env reward sums")
    assert total == env_order_sum(rs), f"{ctx}: total"
    assert np.any(rs != np.round(rs)), f"{ctx}: linear rewards should not sum to integers"


@pytest.mark.parametrize("n_agents,kw", [
    ([64], dict(start_spread=10, reward_mode="linear")),
    ([100], dict(start_spread=12, reward_mode="linear", coord="cartesian")),          # 2 waves
    ([150, 150], dict(start_spread=18, reward_mode="linear", targets=[0] * 150 + [1] * 150)),  # 5 waves -> 8
])
def test_linear_reward_sums_per_step_launch(n_agents, kw):
    E = 5
    targets = kw.pop("targets", None)
    vec, orc = make_pair(E, n_agents, seed=sum(n_agents), targets=targets, **kw)
    check_rollout(vec, orc, 40, np.random.default_rng(sum(n_agents)), state_every=20)
    per_env, _ = vec.reward_sums()
    assert np.any(per_env != np.round(per_env))


@pytest.mark.parametrize("N,E", [(64, 48), (128, 1024)])
def test_linear_reward_sums_rollout_launch(N, E):
    """One rollout launch (the wave kernel's K-step loop; at N = 128 and 1024 envs the workgroup
    path's two env slices on streams of their own) against K oracle steps."""
    K = 12
    vec, orc = make_pair(E, [N], seed=N + E, start_spread=N / 6.0, reward_mode="linear")
    rng = np.random.default_rng(N)
    acts = np.stack([rand_actions(rng, E, N) for _ in range(K)])
    vec.world.reset_counters()
    vec.rollout(torch.from_numpy(acts).cuda())
    rs = np.zeros(E, np.float64)
    for k in range(K):
        rs += pairwise_reward_sum(orc.step(acts[k], n_threads=16)["reward"])
    torch.cuda.synchronize()
    assert vec.status() == 0
    assert_sums(vec, rs, f"rollout N={N}")


@pytest.mark.parametrize("N", [64, 100])
def test_linear_reward_sums_forced_spill(N):
    E = 4
    vec, orc = make_pair(E, [N], seed=N + 1, start_spread=N / 8.0, reward_mode="linear")
    vec.world.set_debug(_abi.DEBUG_FORCE_SPILL)
    check_rollout(vec, orc, 25, np.random.default_rng(N), state_every=25)
    assert vec.spilled() == 25 * E


def test_trajectory_rewards_sum_to_the_counters_at_the_metric_size():
    """4096 x 64, 20 steps in one trajectory launch (bench.py's form): the sums equal the pairwise
    sums of the [K, E, N] rewards the launch returned, row by row; binary mode there, so the total is
    also the positive count minus the collided count."""
    E, N, K = 4096, 64, 20
    vec = FlockVec(E, n_agents=[N], seed=0x6D61636D, device="cuda:0")
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(5)
    acts = torch.randint(0, 3, (K, E, N, 3), dtype=torch.uint8, device="cuda:0", generator=gen)
    vec.world.reset_counters()
    traj = vec.rollout(acts, trajectory=True)
    rew = traj["reward"].cpu().numpy()
    rs = np.zeros(E, np.float64)
    for k in range(K):
        rs += pairwise_reward_sum(rew[k])
    per_env, total = vec.reward_sums()
    np.testing.assert_array_equal(per_env, rs)
    c = vec.counters()
    assert total == env_order_sum(rs) == float(c[2] - c[1])


def test_closed_loop_linear_reward_sums():
    """The closed loop with the device bot (rollout_bots): the trajectory's rewards summed in order."""
    E, N, K = 64, 64, 30
    vec = FlockVec(E, n_agents=[N], seed=9, device="cuda:0", reward_mode="linear")
    from gym_macm.bots import flock_actions
    acts = torch.empty((K + 1, E, N, 3), dtype=torch.uint8, device="cuda:0")
    acts[0] = flock_actions(vec.obs)
    vec.world.reset_counters()
    traj = vec.rollout_bots(acts, K, trajectory=True)
    rew = traj["reward"].cpu().numpy()
    rs = np.zeros(E, np.float64)
    for k in range(K):
        rs += pairwise_reward_sum(rew[k])
    assert_sums(vec, rs, "closed loop")


def test_reset_counters_zeroes_the_sums():
    vec = FlockVec(4, n_agents=[16], seed=3, device="cuda:0", start_spread=4, reward_mode="linear")
    vec.step(torch.ones((4, 16, 3), dtype=torch.uint8, device="cuda:0"))
    per_env, total = vec.reward_sums()
    assert np.any(per_env != 0.0)
    vec.world.reset_counters()
    per_env, total = vec.reward_sums()
    assert total == 0.0 and not per_env.any()
