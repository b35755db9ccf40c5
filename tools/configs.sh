#!/bin/bash
# Throughput at every BASELINE.json config on 1 GPU, each with its bounded CPU-oracle
# baseline (same E x N, ~15 s of CPU work), plus the closed-loop bots runs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-cfg}
mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; return $rc; }
run m_4096x64 --steps 1000 --warmup 100 && \
run c2_1024x64 --envs 1024 --agents 64 --steps 300 --warmup 30 && \
run c3_4096x256_4flocks --envs 4096 --agents 256 --flocks 4 --steps 60 --warmup 5 && \
run c4_tdm_4096x2x16 --env tdm --steps 1000 --warmup 100 && \
run c5_2048x1024 --envs 2048 --agents 1024 --steps 6 --warmup 2 && \
run m_bots_closed_loop --policy bots --steps 300 --warmup 300 --no-cpu-baseline && \
run c4_tdm_bots_closed_loop --env tdm --policy bots --steps 300 --warmup 30 --no-cpu-baseline
