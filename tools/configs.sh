#!/bin/bash
# Throughput at the BASELINE.json configs other than the headline one (1 GPU).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-cfg}
mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; return $rc; }
run c2_1024x64 --envs 1024 --agents 64 --steps 300 --warmup 30 && \
run c3_4096x256_4flocks --envs 4096 --agents 256 --flocks 4 --steps 60 --warmup 5 && \
run c5_2048x1024 --envs 2048 --agents 1024 --steps 6 --warmup 2
