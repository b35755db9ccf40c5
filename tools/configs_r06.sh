#!/bin/bash
# Every BASELINE.json config on 1 GPU in the driver's window (W = 5, K = 20 from reset) and at steady
# state, each with its bounded CPU-oracle baseline (and so the chain floor), the closed loops, the
# overwrite outputs form, and the worlds above 1024 agents (round 6 table, with the C4 per-GPU shard and C2 in the window).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-cfg_r06}
mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; return $rc; }
run m_window --steps 20 --warmup 5 && \
run m_overwrite_window --steps 20 --warmup 5 --outputs overwrite --no-cpu-baseline && \
run m_steady --steps 1000 --warmup 100 --no-cpu-baseline && \
run m_f64_window --steps 20 --warmup 5 --obs-f64 --no-cpu-baseline && \
run c2_window --envs 1024 --agents 64 --steps 20 --warmup 5 && \
run c2_steady --envs 1024 --agents 64 --steps 1000 --warmup 100 && \
run c3_window --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
run c3_steady --envs 4096 --agents 256 --flocks 4 --steps 100 --warmup 50 --no-cpu-baseline && \
run c4_window --env tdm --steps 20 --warmup 5 && \
run c4_steady --env tdm --steps 1000 --warmup 100 --no-cpu-baseline && \
run c4_512_window --env tdm --envs 512 --steps 20 --warmup 5 && \
run c4_512_steady --env tdm --envs 512 --steps 1000 --warmup 100 --no-cpu-baseline && \
run c5_window --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
run c5_steady --envs 2048 --agents 1024 --steps 10 --warmup 100 --no-cpu-baseline && \
run m_bots --policy bots --steps 100 --warmup 300 --no-cpu-baseline && \
run c4_bots --env tdm --policy bots --steps 100 --warmup 100 --no-cpu-baseline && \
run c3_bots --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200 --no-cpu-baseline && \
run big2048_window --envs 256 --agents 2048 --steps 10 --warmup 2 && \
run big4096_window --envs 64 --agents 4096 --steps 5 --warmup 2 --no-cpu-baseline && \
run tdm_big_window --env tdm --teams 1024,1024 --envs 128 --steps 10 --warmup 2 --no-cpu-baseline
