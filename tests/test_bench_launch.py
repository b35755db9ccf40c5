"""bench.py's `--gpus N` against the launcher, on CPU through the --dry-run hook
(launch, gloo process group, shard split, counter all-reduce; no device work):

- `python bench.py --gpus 2` with no launcher environment starts two ranks itself (torch.distributed.run
  as a child process) and reports n_gpus 2 with two shards;
- under a launcher, a --gpus that disagrees with WORLD_SIZE is refused;
- --gpus 1 / no flag stays one process.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _clean_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


def _line(p):
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    return json.loads(lines[0])


def test_gpus_2_without_launcher_starts_two_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo", "--dry-run", "--envs", "8"],
                       capture_output=True, text=True, timeout=240, env=_clean_env(), cwd=REPO)
    d = _line(p)
    assert d["n_gpus"] == 2 and d["ranks_reporting"] == 2
    assert d["config"]["shards"] == [[0, 8], [8, 8]] and d["config"]["total_envs"] == 16


def test_gpus_2_strong_split_without_launcher():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo", "--dry-run",
                        "--total-envs", "301"], capture_output=True, text=True, timeout=240, env=_clean_env(), cwd=REPO)
    d = _line(p)
    assert d["n_gpus"] == 2 and d["config"]["shards"] == [[0, 151], [151, 150]] and d["config"]["total_envs"] == 301


def test_launcher_world_disagreeing_with_gpus_is_refused():
    env = _clean_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29577")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=REPO)
    assert p.returncode != 0 and "must agree" in p.stderr


def test_single_process_default():
    for extra in ([], ["--gpus", "1"]):
        p = subprocess.run([sys.executable, BENCH, "--dry-run", "--envs", "4096"] + extra, capture_output=True,
                           text=True, timeout=120, env=_clean_env(), cwd=REPO)
        d = _line(p)
        assert d["n_gpus"] == 1 and d["config"]["shards"] == [[0, 4096]]
        assert "torch.distributed.run" not in p.stderr
