#!/bin/bash
# Round-4 box session: kernel A's one-thread island walks with the next edge read ahead, and the
# big-island threshold with it (parity subset + A/B).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04p}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_islands.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_grid.py tests/test_gpu_wide_levels.py tests/test_gpu_bots.py tests/test_gpu_tdm.py > "$OUT/pytest.log" 2>&1; st pytest $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c3bots:shd,spf,spf96,spf200 c3:shd,spf,spf96 mbots:spf,wbf c4bots:spf,wbf" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
