#!/bin/bash
# Round-4 box session: the rollout with an opaque lane index (no hoisted lane-derived values; the
# TDM rollout's scratch spill gone): parity subset, A/B, and C4 PMC traffic before / after.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04r}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_rollout.py tests/test_gpu_tdm.py tests/test_gpu_headline.py tests/test_gpu_bots.py \
  tests/test_gpu_trajectory.py tests/test_gpu_tdm_spill.py > "$OUT/pytest.log" 2>&1; st pytest $?
for v in fin2 rol1; do
  MACM_LIB="$R/ab/$v.so" timeout -k 10 300 bash tools/pmc.sh "$OUT/pmc_c4_$v" --env tdm --steps 20 --warmup 5 \
    > "$OUT/pmc_c4_$v.log" 2>&1; st "pmc_c4_$v" $?
done
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c4:fin2,rol1 c4bots:fin2,rol1 mtr:rol1,rol2 mss:rol1,rol2 mbots:rol1,rol2" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
