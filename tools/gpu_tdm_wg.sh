#!/bin/bash
# The TDM workgroup-step tests, then (if green) the whole GPU suite. Each step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-tdm_wg}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_tdm_wg.py -m gpu -x -v -rf --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_tdm_wg.log" 2>&1; rc=$?
echo "tdm_wg rc=$rc" | tee "$OUT/status.txt"
[ $rc -eq 0 ] || exit $rc
[ "${FULL:-1}" = 1 ] || exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "full rc=$rc" | tee -a "$OUT/status.txt"
exit $rc
