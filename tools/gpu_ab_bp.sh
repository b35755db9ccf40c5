#!/bin/bash
# Kernel B branch-free position level steps: the GPU suite with the tree's library (wave kernel's
# position steps branch-free now), the suite against ab/bp1.so, then an A/B bp0 / bp1.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/bpab; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
MACM_LIB="$PWD/ab/bp1.so" timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_multiproc.py > "$OUT/pytest_bp1.log" 2>&1 || { echo "pytest bp1 rc=$?"; tail -30 "$OUT/pytest_bp1.log"; exit 1; }
tail -1 "$OUT/pytest_bp1.log"
bash tools/ab_set.sh bpab "c5 c3bots c3" ab/bp0.so ab/bp1.so && python tools/ab_set_summary.py gpurun_out/bpab
