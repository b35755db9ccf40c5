#!/bin/bash
# Round-4 box session: the nearest-neighbour ring expansion of the strip cells (parity + A/B), and
# the uniform-register level-step microbenchmark.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04i}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_grid.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_islands.py \
  > "$OUT/pytest.log" 2>&1; st pytest $?
timeout -k 10 300 tools/build/ubench_level > "$OUT/ubench_level.txt" 2>&1; st ubench $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c3bots:walk,ring,ring512 c3:walk,ring,ring512" > "$OUT/ab.log" 2>&1; st ab $?
bash tools/phase_wg.sh "$(basename $OUT)/phase" ring > "$OUT/phase.log" 2>&1; st phase $?
echo ALLDONE | tee -a "$OUT/status.txt"
