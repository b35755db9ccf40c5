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
    rewards = []
    for t in range(STEPS):
        r = orc.step(acts[t])
        ctr += gdist.step_counters(r["reward"], r["collided"], r["done"])
        rewards.append(r["reward"])
    total = gdist.reduce_counters(ctr)
    slowest = gdist.reduce_max(float(rank + 1))
    np.save(os.path.join(outdir, f"rank{rank}_rewards.npy"), np.stack(rewards))
    np.save(os.path.join(outdir, f"rank{rank}_total.npy"), total)
    np.save(os.path.join(outdir, f"rank{rank}_max.npy"), np.array([slowest]))
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
    rewards = []
    for t in range(STEPS):
        r = full.step(acts[t])
        ctr += gdist.step_counters(r["reward"], r["collided"], r["done"])
        rewards.append(r["reward"])
    rewards = np.stack(rewards)
    for rank in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"rank{rank}_rewards.npy"),
                                      rewards[:, gdist.shard_slice(rank, E_PER_RANK)])
        np.testing.assert_array_equal(np.load(tmp_path / f"rank{rank}_total.npy"), ctr)
        assert float(np.load(tmp_path / f"rank{rank}_max.npy")[0]) == 2.0
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
