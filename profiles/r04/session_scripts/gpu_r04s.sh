#!/bin/bash
# Round-4 box session: TDM obs in row-block order (parity, PMC traffic, A/B).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04s}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_tdm.py tests/test_gpu_tdm_spill.py tests/test_gpu_tdm_wg.py tests/test_gpu_bots.py \
  tests/test_gpu_fullsize.py tests/test_gpu_rollout.py tests/test_gpu_trajectory.py > "$OUT/pytest.log" 2>&1; st pytest $?
MACM_LIB="$R/ab/rb.so" timeout -k 10 300 bash tools/pmc.sh "$OUT/pmc_c4_rb" --env tdm --steps 20 --warmup 5 \
  > "$OUT/pmc_c4_rb.log" 2>&1; st pmc_c4_rb $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c4:rol1,rb c4bots:rol1,rb" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
