#!/bin/bash
# Every BASELINE.json config on 1 GPU in the driver's window (W = 5, K = 20 from reset) and at steady
# state, each with its bounded CPU-oracle baseline, plus the closed-loop bots runs (round 4 table).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-cfg_r04}
mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; return $rc; }
run m_window --steps 20 --warmup 5 && \
run m_steady --steps 1000 --warmup 100 --no-cpu-baseline && \
run m_f64_window --steps 20 --warmup 5 --obs-f64 --no-cpu-baseline && \
run m_traj_window --steps 20 --warmup 5 --trajectory --no-cpu-baseline && \
run c2_steady --envs 1024 --agents 64 --steps 1000 --warmup 100 && \
run c3_window --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
run c3_steady --envs 4096 --agents 256 --flocks 4 --steps 100 --warmup 50 --no-cpu-baseline && \
run c4_window --env tdm --steps 20 --warmup 5 && \
run c4_steady --env tdm --steps 1000 --warmup 100 --no-cpu-baseline && \
run c5_window --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
run c5_steady --envs 2048 --agents 1024 --steps 10 --warmup 100 --no-cpu-baseline && \
run m_bots --policy bots --steps 100 --warmup 300 --no-cpu-baseline && \
run c4_bots --env tdm --policy bots --steps 100 --warmup 100 --no-cpu-baseline && \
run c3_bots --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200 --no-cpu-baseline
