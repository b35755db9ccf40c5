"""bench.py's multi-process path on the GPU box: two ranks under torchrun (one process each,
both on the box's one GPU, gloo for the counter all-reduce since RCCL needs one GPU per rank).
Each rank steps its own shard of global env ids; the reduced counters must cover both shards
and the line must report the whole job. The RCCL flavour (`--dist-backend nccl`, the default) needs one GPU
per rank, so on this box it runs as one rank under torchrun (test_rccl_single_rank_under_torchrun);
its multi-rank form runs in the driver's 8-GPU scaling bench."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("env,extra", [("flock", []), ("tdm", ["--env", "tdm"]),
                                        ("flock_wg", ["--agents", "100"])])
def test_two_ranks_sharded_bench(env, extra):
    E, K, W = 128, 6, 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", str(K), "--warmup", str(W), "--envs", str(E), "--dist-backend", "gloo",
           "--no-cpu-baseline"] + extra
    env_vars = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env_vars, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == K and d["warmup"] == W
    N = d["config"]["n_agents"]
    assert d["config"]["total_envs"] == 2 * E
    if env != "tdm":
        assert d["counters"]["agent_steps"] == 2 * E * N * K
    assert d["value"] > 0 and d["ms_per_step"] > 0


def test_gpus_2_without_launcher_runs_two_ranks():
    """`python bench.py --gpus 2` with no launcher environment: bench.py starts the two
    ranks itself as a child torch.distributed.run before touching the GPU; both step their shard on
    the box's one GPU (gloo counters) and the line reports the whole job."""
    E, K, W = 128, 4, 2
    env_vars = {k: v for k, v in os.environ.items()
                if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env_vars.update(HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", str(K), "--warmup", str(W),
           "--envs", str(E), "--dist-backend", "gloo", "--no-cpu-baseline"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env_vars, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["shards"] == [[0, E], [E, E]]
    assert d["counters"]["agent_steps"] == 2 * E * d["config"]["n_agents"] * K


def _run(cmd):
    env_vars = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env_vars, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("extra", [[], ["--agents", "100"]])
def test_strong_split_two_ranks_equal_single_process(tmp_path, extra):
    """bench.py --total-envs T (BASELINE configs 4 and 5 name totals: 4096 / 16384 envs over 8 GPUs):
    2 ranks take contiguous shares of T = 301 envs (151 + 150), the actions are the whole job's draw,
    so every env's final state equals the single-process run of all 301 envs, bit for bit, and the
    reduced counters equal its counters."""
    import numpy as np
    T, K, W = 301, 6, 2
    base = [os.path.join(REPO, "bench.py"), "--steps", str(K), "--warmup", str(W), "--total-envs", str(T),
            "--no-cpu-baseline"] + extra
    one = _run([sys.executable] + base + ["--dump-final", str(tmp_path / "one")])
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + base +
               ["--gpus", "2", "--dist-backend", "gloo", "--dump-final", str(tmp_path / "two")])
    for d in (one, two):
        assert d["scaling"] == "strong" and d["config"]["total_envs"] == T
    assert two["counters"] == one["counters"]
    ref = np.load(tmp_path / "one.rank0.npz")
    seen = 0
    for r in range(2):
        part = np.load(tmp_path / f"two.rank{r}.npz")
        o = int(part["env_offset"])
        n = part["pos"].shape[0]
        assert (o, n) == ((0, 151) if r == 0 else (151, 150))
        for k in ("pos", "vel", "angle", "fat", "sleep", "contact_count", "step_count", "time_passed"):
            np.testing.assert_array_equal(part[k], ref[k][o:o + n], err_msg=f"rank {r} {k}")
        for k in ("contact_ab", "contact_imp"):  # rows of max(contact_count) entries (World.get_state)
            w = max(part[k].shape[1], ref[k].shape[1])
            pad = lambda a: np.concatenate([a, np.zeros((a.shape[0], w - a.shape[1]) + a.shape[2:], a.dtype)], 1)
            np.testing.assert_array_equal(pad(part[k]), pad(ref[k][o:o + n]), err_msg=f"rank {r} {k}")
        seen += n
    assert seen == T


@pytest.mark.parametrize("extra", [[], ["--agents", "100"]])
def test_rccl_single_rank_under_torchrun(extra):
    """The RCCL branch of bench.py (`--dist-backend nccl`, the default) on the one-GPU box: torchrun
    with one rank creates the nccl (= RCCL) process group, and the barriers around the timed window
    and the device-tensor all-reduces of the counters and the elapsed time run through RCCL. The
    reduced counters equal the plain single-process run's (same envs, same actions)."""
    K, W, E = 4, 2, 96
    base = [os.path.join(REPO, "bench.py"), "--steps", str(K), "--warmup", str(W), "--envs", str(E),
            "--no-cpu-baseline"] + extra
    one = _run([sys.executable] + base)
    rccl = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                 "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + base +
                ["--gpus", "1", "--dist-backend", "nccl"])
    assert "RCCL counters" in rccl["config"]["parallelism"]
    assert "RCCL" not in one["config"]["parallelism"]
    assert rccl["counters"] == one["counters"]
    assert rccl["n_gpus"] == 1 and rccl["value"] > 0
