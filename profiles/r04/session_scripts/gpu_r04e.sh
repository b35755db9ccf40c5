#!/bin/bash
# Round-4: microbenchmark (fixed chain-lane prefetch, unrolled form) and the workgroup-path parity
# tests against the kernel-B level-loop rewrite.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04e}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 5 120 tools/build/ubench_level > "$OUT/ubench_level.txt" 2>&1; st ubench $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_islands.py tests/test_gpu_grid.py \
  tests/test_gpu_dense.py tests/test_gpu_rollout.py tests/test_gpu_headline.py \
  > "$OUT/pytest.log" 2>&1; st pytest $?
echo ALLDONE | tee -a "$OUT/status.txt"
