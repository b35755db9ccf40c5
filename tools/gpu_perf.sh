#!/bin/bash
# GPU perf iteration: full GPU tests, Flock + TDM benches (no CPU baseline), rocprofv3 stats of the Flock bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${OUT_NAME:-perf}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc" | tee "$OUT/status.txt"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > "$OUT/bench_flock.json" 2> "$OUT/bench_flock.err" || exit $?
timeout -k 10 300 python bench.py --env tdm --steps 1000 --warmup 100 --no-cpu-baseline > "$OUT/bench_tdm.json" 2> "$OUT/bench_tdm.err" || exit $?
timeout -k 10 300 python bench.py --policy bots --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/bench_flock_bots.json" 2> "$OUT/bench_flock_bots.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err" || exit $?
echo ALLDONE | tee -a "$GRAFT_REPO_ROOT/$OUT/status.txt"
