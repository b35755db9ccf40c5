"""Env-sharded multi-GPU helpers (one process per GPU, torch.distributed).

The reference has no parallelism at all (one Box2D world per env, single thread;
SURVEY.md §2). Its envs are fully independent, so the MI355X layout is weak
scaling with no data-path collective: rank r owns the contiguous global env ids
[r*E, (r+1)*E), and because every env is seeded by its GLOBAL id (env e ==
Flock after random.seed(seed + e)) its trajectory is identical whatever the
number of ranks. The only collectives are one small all-reduce of counters after
a measurement window and one all-gather of the per-env reward sums (RCCL over
xGMI when backend="nccl", gloo in CPU tests).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def rank_info():
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def env_offset(rank: int, envs_per_rank: int) -> int:
    """First global env id of `rank` under weak scaling."""
    return rank * envs_per_rank


def shard_slice(rank: int, envs_per_rank: int) -> slice:
    o = env_offset(rank, envs_per_rank)
    return slice(o, o + envs_per_rank)


def strong_split(total_envs: int, world: int, rank: int):
    """(first global env id, env count) of `rank` when `total_envs` are split over `world` ranks
    (strong scaling, e.g. BASELINE config 4: 4096 envs over 8 GPUs; config 5: 16384 over 8):
    contiguous shards, the first total_envs % world ranks one env larger."""
    base, extra = divmod(int(total_envs), int(world))
    count = base + (1 if rank < extra else 0)
    return rank * base + min(rank, extra), count


def reduce_counters(counters, device=None, op="sum"):
    """All-reduce an int64 counter vector across ranks (no-op without a process group)."""
    t = torch.as_tensor(np.asarray(counters, np.int64), dtype=torch.int64)
    if device is not None:
        t = t.to(device)
    if dist.is_available() and dist.is_initialized():  # one rank too: the collective still runs
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
    return t.cpu().numpy()


def reduce_max(value: float, device=None) -> float:
    """Max over ranks (the job's wall time is its slowest rank's)."""
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def step_counters(reward: np.ndarray, collided: np.ndarray, done: np.ndarray) -> np.ndarray:
    """Host-side counters of one step with the device counters' meaning
    (macm_world_counters): agent-steps, collided agent-steps, positive-reward
    agent-steps, env-steps with done set."""
    return np.array([reward.size, int(collided.sum()), int((reward > 0).sum()), int(done.sum())], np.int64)


def pairwise_reward_sum(reward: np.ndarray) -> np.ndarray:
    """One step's reward sum per env in the device's order (macm_world_reward_sums, flock_common.hpp
    block_pairwise_sum): the float32 rewards [E, N] as float64, summed pairwise over the agent slots
    0 .. P-1 with +0.0 past N, P = 64 * 2^ceil(log2(ceil(N / 64))): ((r0 + r1) + (r2 + r3)) + ...
    Returns [E] float64. The per-env total is these sums added in step order from +0.0."""
    r = np.asarray(reward, np.float32).astype(np.float64)
    E, N = r.shape
    waves = -(-N // 64)
    n2 = 1
    while n2 < waves:
        n2 <<= 1
    x = np.zeros((E, 64 * n2), np.float64)
    x[:, :N] = r
    while x.shape[1] > 1:
        x = x[:, 0::2] + x[:, 1::2]
    return x[:, 0]


def env_order_sum(values) -> float:
    """Sum in the given order from +0.0, one IEEE addition at a time (macm_world_reward_sums'
    total; numpy's sum is pairwise, which would differ in the last bits)."""
    acc = 0.0
    for v in np.asarray(values, np.float64).tolist():
        acc += v
    return acc


def reduce_reward_sums(per_env, device=None) -> float:
    """The job's reward total from every rank's per-env totals: gathered in rank order (ranks own
    contiguous, increasing global env ranges in both the weak and the strong split) and summed in
    global env order, so the total is bit-identical to a single-process run of the whole job at any
    rank count (an all-reduce would add the ranks' partial sums in a topology-dependent order)."""
    x = np.asarray(per_env, np.float64).reshape(-1)
    if not (dist.is_available() and dist.is_initialized()):
        return env_order_sum(x)
    world = dist.get_world_size()
    n = torch.tensor([x.size], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(t.item()) for t in sizes]
    m = max(sizes)
    buf = torch.zeros((m,), dtype=torch.float64, device=device)
    buf[:x.size] = torch.from_numpy(x).to(buf.device)
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    allv = np.concatenate([p.cpu().numpy()[:k] for p, k in zip(parts, sizes)])
    return env_order_sum(allv)
