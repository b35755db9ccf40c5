#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r01}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
stop_if_crash() {  # $1 = exit code, $2 = step name; pytest 1 = test failures (not a crash)
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP: $2 exited $rc" | tee -a "$OUT/status.txt"; exit "$rc"; fi
  echo "$2 rc=$rc" | tee -a "$OUT/status.txt"
}
nproc > "$OUT/host.txt"; lscpu | grep -i "model name" >> "$OUT/host.txt"; rocm-smi --showproductname >> "$OUT/host.txt" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
stop_if_crash $? pytest_gpu
timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1
stop_if_crash $? smoke
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > "$OUT/bench.json" 2> "$OUT/bench.err"
stop_if_crash $? bench
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
stop_if_crash $? rocprof
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --env tdm --steps 300 --warmup 30 > "$OUT/bench_tdm.json" 2> "$OUT/bench_tdm.err"
stop_if_crash $? bench_tdm
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_tdm" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --env tdm --steps 200 --warmup 20 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_tdm_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof_tdm.err"
stop_if_crash $? rocprof_tdm
echo ALLDONE | tee -a "$GRAFT_REPO_ROOT/$OUT/status.txt"
