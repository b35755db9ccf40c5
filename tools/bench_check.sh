#!/bin/bash
# bench.py lines of the round: the driver's default window, --obs-f64, TDM, C3 (4 flocks), C5.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-bc}
mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; return $rc; }
run m_w5 --steps 20 --warmup 5 && \
run m_w5_f64 --steps 20 --warmup 5 --obs-f64 && \
run m_1000 --steps 1000 --warmup 100 && \
run c4_w5 --env tdm --steps 20 --warmup 5 && \
run c3_w5 --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
run c5_w5 --envs 2048 --agents 1024 --steps 20 --warmup 5 && \
echo ALLDONE
