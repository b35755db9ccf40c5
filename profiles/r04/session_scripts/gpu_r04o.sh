#!/bin/bash
# Round-4 box session: shared dummy slot in the level steps (kernel B and the wave kernel's
# one-slot path), wide-level issue priority; parity subset + A/B.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04o}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_headline.py tests/test_gpu_wide_levels.py \
  tests/test_gpu_islands.py tests/test_gpu_dense.py > "$OUT/pytest.log" 2>&1; st pytest $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c5r:head,shd c3bots:head,shd mtr:head,shd mbots:head,shd,wprio" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
