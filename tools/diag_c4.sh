#!/bin/bash
# Round 6 diagnostic (wrong results by design): where the fused TDM observation's time goes at full
# occupancy: v0 shipped, v1 without the atan2 core, v2 without the row-block obs / mask global stores.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-diag_c4}
mkdir -p "$OUT"
LIBS=(abv/final.so abv/d_noatan.so abv/d_nostore.so)
for r in 1 2 3; do
  for i in 0 1 2; do
    MACM_TDM_TAIL_OBS=0 MACM_TDM_SPLIT_OBS=0 MACM_LIB="$PWD/${LIBS[$i]}" timeout -k 10 200 python bench.py --no-cpu-baseline --env tdm --steps 20 --warmup 5 > "$OUT/c4_window_v${i}_r$r.json" 2> "$OUT/c4_window_v${i}_r$r.err" || exit $?
    MACM_TDM_TAIL_OBS=0 MACM_TDM_SPLIT_OBS=0 MACM_LIB="$PWD/${LIBS[$i]}" timeout -k 10 200 python bench.py --no-cpu-baseline --env tdm --envs 512 --steps 20 --warmup 5 > "$OUT/c4_512_fused_window_v${i}_r$r.json" 2> "$OUT/c4_512_fused_window_v${i}_r$r.err" || exit $?
  done
done
echo ALLDONE
