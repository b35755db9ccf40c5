#!/bin/bash
# End-of-iteration GPU evidence in one session: parity tests, smoke, rocprofv3 kernel stats
# (Flock, TDM), PMC passes (Flock, TDM) and their summaries, the metric benches with their CPU
# baselines (traffic from those summaries) and every BASELINE config. Each GPU step has its own time limit; a crash or timeout ends the script.
#   tools/gpu_final.sh OUTNAME      -> gpurun_out/OUTNAME/
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
NAME=${1:-final}
OUT=gpurun_out/$NAME
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
stop() { local rc=$1; echo "$2 rc=$rc" | tee -a "$OUT/status.txt"; [ "$rc" -eq 0 ] || exit "$rc"; }
{ nproc; lscpu | grep -i "model name"; rocm-smi --showproductname; } > "$OUT/host.txt" 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
stop $? pytest_gpu
timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1
stop $? smoke
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1000 --warmup 100 \
    --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err" )
stop $? rocprof_flock
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/$OUT/prof_tdm" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --env tdm --steps 1000 \
    --warmup 100 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_tdm_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof_tdm.err" )
stop $? rocprof_tdm
bash tools/pmc.sh "$OUT/pmc_flock" --steps 200 --warmup 20 > "$OUT/pmc_flock.log" 2>&1
stop $? pmc_flock
bash tools/pmc.sh "$OUT/pmc_tdm" --env tdm --steps 200 --warmup 20 > "$OUT/pmc_tdm.log" 2>&1
stop $? pmc_tdm
# the PMC summaries of this session feed the bench lines' roofline.traffic (copy them to profiles/)
python tools/pmc_summary.py "$OUT/pmc_flock" --envs 4096 --agents 64 -o "$OUT/pmc_flock_step.json" > "$OUT/pmc_summary.log" 2>&1
stop $? pmc_summary_flock
python tools/pmc_summary.py "$OUT/pmc_tdm" --kernel "env_step_w64<1, 32, float, false>" --envs 4096 --agents 32 \
    -o "$OUT/pmc_tdm_step.json" >> "$OUT/pmc_summary.log" 2>&1
stop $? pmc_summary_tdm
timeout -k 10 300 python bench.py --traffic-json "$OUT/pmc_flock_step.json" > "$OUT/bench.json" 2> "$OUT/bench.err"
stop $? bench
timeout -k 10 300 python bench.py --env tdm --traffic-json "$OUT/pmc_tdm_step.json" > "$OUT/bench_tdm.json" 2> "$OUT/bench_tdm.err"
stop $? bench_tdm
bash tools/configs.sh "$NAME/configs" > "$OUT/configs.log" 2>&1
stop $? configs
echo ALLDONE | tee -a "$OUT/status.txt"
