#!/bin/bash
# pytest -m gpu on the selected files (args; default: all), then optional C3/C5 benches.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${OUT_NAME:-t}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc" | tee "$OUT/status.txt"
[ $rc -eq 0 ] || exit $rc
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 300 python bench.py --envs 4096 --agents 256 --flocks 4 --steps 60 --warmup 5 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err" || exit $?
timeout -k 10 300 python bench.py --envs 2048 --agents 1024 --steps 6 --warmup 2 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" || exit $?
timeout -k 10 300 python bench.py --policy bots --envs 4096 --agents 256 --flocks 4 --steps 100 --warmup 200 --no-cpu-baseline > "$OUT/c3_bots.json" 2> "$OUT/c3_bots.err" || exit $?
fi
echo ALLDONE | tee -a "$OUT/status.txt"
