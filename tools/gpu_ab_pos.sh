#!/bin/bash
# Round-3 A/B: the position passes' island-minimum atomics inside each level step (posold) vs once
# after the level loop (posnew, the product default); the GPU tests first (bit-exactness of the change).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
OUT=gpurun_out/posab; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
bash tools/ab_set.sh posab "c5 c3bots mbots mtr" ab/posold.so ab/posnew.so && python tools/ab_set_summary.py gpurun_out/posab
