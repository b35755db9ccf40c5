#!/bin/bash
# Round-4 box session: kernel C's pipelined candidate loop, the DFS record batch, the big-island
# threshold with the faster serial walk.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04j}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_grid.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_islands.py \
  > "$OUT/pytest.log" 2>&1; st pytest $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c5r:ring,pipe0,pipe1,pipe2,b8 c3:ring,pipe1,pipe2,big96,big4k c3bots:ring,pipe1,big96,big4k" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
