#!/bin/bash
# Round-4 box session: the wave kernel's TDM hand-over takes its spill slot before committing
# (TDM spill / pooled-slot tests), then C4 timings against the committed library.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04v}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_tdm_spill.py tests/test_gpu_tdm.py tests/test_gpu_tdm_wg.py tests/test_gpu_dense.py > "$OUT/pytest.log" 2>&1; st pytest $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c4:rb3,slotfix" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
