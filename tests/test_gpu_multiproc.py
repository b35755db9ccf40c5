"""bench.py's multi-process path on the GPU box: two ranks under torchrun (one process each,
both on the box's one GPU, gloo for the counter all-reduce since RCCL needs one GPU per rank).
Each rank steps its own shard of global env ids; the reduced counters must cover both shards
and the line must report the whole job. The RCCL flavour of the same code runs in the driver's
8-GPU scaling bench (`--dist-backend nccl`, the default)."""
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
