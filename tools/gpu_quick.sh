#!/bin/bash
# Quick GPU check: selected pytest files (args) + short TDM/Flock closed-loop benches.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${OUT_NAME:-quick}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest "$@" -q -rf > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc" | tee "$OUT/status.txt"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --policy bots --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/bench_flock_bots.json" 2> "$OUT/bench_flock_bots.err" || exit $?
timeout -k 10 300 python bench.py --env tdm --policy bots --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/bench_tdm_bots.json" 2> "$OUT/bench_tdm_bots.err" || exit $?
echo ALLDONE | tee -a "$OUT/status.txt"
