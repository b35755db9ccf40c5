#!/bin/bash
# GPU tests with the tree's library (the candidate change), then an A/B of library variants:
#   tools/gpu_ab_tests.sh OUTNAME "workloads" ab/v0.so ab/v1.so ...
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
NAME=$1; WL=$2; shift 2
OUT=gpurun_out/$NAME; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash tools/ab_set.sh "$NAME" "$WL" "$@" && python tools/ab_set_summary.py "gpurun_out/$NAME"
