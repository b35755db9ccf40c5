#!/bin/bash
# Wave-kernel branch-free level steps: the whole GPU suite against ab/wl2.so (velocity + position
# passes branch-free; the tree's library has the velocity passes only and passed the suite), then
# an A/B of wl0 (exec-masked steps) / wl1 (velocity branch-free) / wl2 (both).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/wlab; mkdir -p "$OUT"
MACM_LIB="$PWD/ab/wl2.so" timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_multiproc.py > "$OUT/pytest_wl2.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest_wl2.log"; exit 1; }
tail -1 "$OUT/pytest_wl2.log"
bash tools/ab_set.sh wlab "mtr mbots mss c2" ab/wl0.so ab/wl1.so ab/wl2.so && python tools/ab_set_summary.py gpurun_out/wlab
