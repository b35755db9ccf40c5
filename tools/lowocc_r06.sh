#!/bin/bash
# Round 6: the low-occupancy configs: C4's per-GPU shard (512 envs of 2 x 16) and C2
# (1024 envs x 64), window and steady, beside the 4096-env C4 and M windows of the same session.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-lowocc_r06}
mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; return $rc; }
run c4_512_window --env tdm --envs 512 --steps 20 --warmup 5 --no-cpu-baseline && \
run c4_512_steady --env tdm --envs 512 --steps 1000 --warmup 100 --no-cpu-baseline && \
run c4_window --env tdm --steps 20 --warmup 5 --no-cpu-baseline && \
run c4_steady --env tdm --steps 1000 --warmup 100 --no-cpu-baseline && \
run c2_window --envs 1024 --agents 64 --steps 20 --warmup 5 --no-cpu-baseline && \
run c2_steady --envs 1024 --agents 64 --steps 1000 --warmup 100 --no-cpu-baseline && \
run m_window --steps 20 --warmup 5 --no-cpu-baseline
