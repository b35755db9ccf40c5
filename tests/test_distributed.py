"""Multi-process (gloo, world_size 2, CPU) tests of the env-sharded layout used by
bench.py on N GPUs: each rank steps ONLY its shard (global env ids rank*E ..),
results per env are identical to a single-process run of the whole batch, and the
counter all-reduce equals the single-process totals. The per-rank world here is
the CPU oracle (these tests run without a GPU); the HIP world's shard invariance
is tested in tests/test_gpu_parity.py::test_shard_offsets_are_slices_of_the_full_batch.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

E_PER_RANK, N, STEPS, SEED = 3, 16, 25, 4242


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _config():
    from gym_macm.settings import flockSettings, to_config
    return to_config(flockSettings(start_spread=8), N, 1, obs_f64=True)


def _actions(world):
    rng = np.random.default_rng(7)
    return rng.integers(0, 3, size=(STEPS, world * E_PER_RANK, N, 3)).astype(np.uint8)


def _worker(rank, world, port, outdir):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "gym-macm_amd"), os.path.join(repo, "oracle")]
    import torch.distributed as dist
    from gym_macm import dist as gdist
    from oracle import OracleFlock

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    acts = _actions(world)[:, gdist.shard_slice(rank, E_PER_RANK)]
    orc = OracleFlock(_config(), None, E_PER_RANK, SEED, gdist.env_offset(rank, E_PER_RANK))
    ctr = np.zeros(4, np.int64)
    rs = np.zeros(E_PER_RANK, np.float64)
    rewards = []
    for t in range(STEPS):
        r = orc.step(acts[t])
        ctr += gdist.step_counters(r["reward"], r["collided"], r["done"])
        rs += gdist.pairwise_reward_sum(r["reward"])  # the device's per-env accumulation
        rewards.append(r["reward"])
    total = gdist.reduce_counters(ctr)
    rtotal = gdist.reduce_reward_sums(rs)
    slowest = gdist.reduce_max(float(rank + 1))
    np.save(os.path.join(outdir, f"rank{rank}_rewards.npy"), np.stack(rewards))
    np.save(os.path.join(outdir, f"rank{rank}_total.npy"), total)
    np.save(os.path.join(outdir, f"rank{rank}_max.npy"), np.array([slowest]))
    np.save(os.path.join(outdir, f"rank{rank}_rtotal.npy"), np.array([rtotal]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shards_match_single_process(tmp_path):
    from gym_macm import dist as gdist
    from oracle import OracleFlock

    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    acts = _actions(world)
    full = OracleFlock(_config(), None, world * E_PER_RANK, SEED, 0)
    ctr = np.zeros(4, np.int64)
    rs = np.zeros(world * E_PER_RANK, np.float64)
    rewards = []
    for t in range(STEPS):
        r = full.step(acts[t])
        ctr += gdist.step_counters(r["reward"], r["collided"], r["done"])
        rs += gdist.pairwise_reward_sum(r["reward"])
        rewards.append(r["reward"])
    rewards = np.stack(rewards)
    rtotal = gdist.env_order_sum(rs)
    assert rtotal == float((rewards.astype(np.float32) == 1).sum() - (rewards == -1).sum())  # binary: exact
    for rank in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"rank{rank}_rewards.npy"),
                                      rewards[:, gdist.shard_slice(rank, E_PER_RANK)])
        np.testing.assert_array_equal(np.load(tmp_path / f"rank{rank}_total.npy"), ctr)
        assert float(np.load(tmp_path / f"rank{rank}_max.npy")[0]) == 2.0
        assert float(np.load(tmp_path / f"rank{rank}_rtotal.npy")[0]) == rtotal, f"rank {rank} reward total"
    assert ctr[0] == STEPS * world * E_PER_RANK * N


def test_offsets_partition_global_env_ids():
    from gym_macm import dist as gdist
    ids = np.concatenate([np.arange(4 * 8)[gdist.shard_slice(r, 8)] for r in range(4)])
    np.testing.assert_array_equal(ids, np.arange(32))
    assert gdist.env_offset(3, 4096) == 12288


@pytest.mark.parametrize("total,world", [(4096, 8), (16384, 8), (301, 2), (7, 3), (5, 8)])
def test_strong_split_partitions_the_job(total, world):
    """bench.py --total-envs: contiguous shares covering every global env id once, sizes within 1."""
    from gym_macm import dist as gdist
    parts = [gdist.strong_split(total, world, r) for r in range(world)]
    ids = np.concatenate([np.arange(o, o + n) for o, n in parts])
    np.testing.assert_array_equal(ids, np.arange(total))
    sizes = [n for _, n in parts]
    assert max(sizes) - min(sizes) <= 1


TOTAL8, N8, STEPS8 = 29, 12, 12  # 29 envs over 8 ranks: shards of 4 4 4 4 4 3 3 3


def _strong_config():
    from gym_macm.settings import flockSettings, to_config
    return to_config(flockSettings(start_spread=6, reward_mode="linear"), N8, 1, obs_f64=True)


def _strong_actions():
    rng = np.random.default_rng(11)
    return rng.integers(0, 3, size=(STEPS8, TOTAL8, N8, 3)).astype(np.uint8)


def _strong_worker(rank, world, port, outdir):
    """bench.py --total-envs on `world` ranks, gloo: rank r steps only its contiguous shard
    (gym_macm.dist.strong_split) with the whole job's actions, the counters all-reduced."""
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "gym-macm_amd"), os.path.join(repo, "oracle")]
    import torch.distributed as dist
    from gym_macm import dist as gdist
    from oracle import OracleFlock

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, n = gdist.strong_split(TOTAL8, world, rank)
    acts = _strong_actions()[:, off:off + n]
    orc = OracleFlock(_strong_config(), None, n, SEED, off)
    ctr = np.zeros(4, np.int64)
    rs = np.zeros(n, np.float64)
    for t in range(STEPS8):
        r = orc.step(acts[t])
        ctr += gdist.step_counters(r["reward"], r["collided"], r["done"])
        rs += gdist.pairwise_reward_sum(r["reward"])
    total = gdist.reduce_counters(ctr)
    rtotal = gdist.reduce_reward_sums(rs)
    st = orc.get_state(64 * N8)
    np.savez(os.path.join(outdir, f"strong{rank}.npz"), off=off, n=n, total=total, rtotal=rtotal, pos=st["pos"], vel=st["vel"],
             count=st["contact_count"], ab=st["contact_ab"])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_eight_rank_strong_split_matches_single_process(tmp_path):
    """the strong split the driver's 8-GPU run uses (BASELINE C4: 4096 envs over 8,
    C5: 16,384 over 8) at a reduced, uneven total on 8 gloo ranks: contiguous shards that cover every
    global env once, every env's final state (positions, velocities, the ordered contact list) equal
    to the single-process run of the whole job, and the all-reduced counters equal its totals; the
    linear-mode reward total, gathered per env and summed in global env order, equals the
    single-process total bit for bit."""
    from gym_macm import dist as gdist
    from oracle import OracleFlock

    world = 8
    mp.start_processes(_strong_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    full = OracleFlock(_strong_config(), None, TOTAL8, SEED, 0)
    acts = _strong_actions()
    ctr = np.zeros(4, np.int64)
    rs = np.zeros(TOTAL8, np.float64)
    for t in range(STEPS8):
        r = full.step(acts[t])
        ctr += gdist.step_counters(r["reward"], r["collided"], r["done"])
        rs += gdist.pairwise_reward_sum(r["reward"])
    rtotal = gdist.env_order_sum(rs)
    assert rtotal != round(rtotal), "linear rewards: the total should not be an integer"
    ref = full.get_state(64 * N8)
    seen = []
    for rank in range(world):
        z = np.load(tmp_path / f"strong{rank}.npz")
        off, n = int(z["off"]), int(z["n"])
        assert (off, n) == gdist.strong_split(TOTAL8, world, rank)
        seen += list(range(off, off + n))
        np.testing.assert_array_equal(z["total"], ctr, err_msg=f"rank {rank} all-reduced counters")
        assert float(z["rtotal"]) == rtotal, f"rank {rank} gathered reward total (linear)"
        for k, rk in (("pos", "pos"), ("vel", "vel"), ("count", "contact_count")):
            np.testing.assert_array_equal(z[k], ref[rk][off:off + n], err_msg=f"rank {rank} {k}")
        for e in range(n):
            c = int(z["count"][e])
            np.testing.assert_array_equal(z["ab"][e, :c], ref["contact_ab"][off + e, :c], err_msg=f"env {off + e}")
    assert seen == list(range(TOTAL8))
    assert ctr[0] == STEPS8 * TOTAL8 * N8 and ctr[1] > 0
