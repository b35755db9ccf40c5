#!/bin/bash
# Round-4 box session: trajectory and rollout parity with rollouts of >= 32 steps (balanced order).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04tr}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_trajectory.py tests/test_gpu_rollout.py > "$OUT/pytest.log" 2>&1; st pytest $?
echo ALLDONE | tee -a "$OUT/status.txt"
