#!/bin/bash
# Round 6 diagnostic (wrong masks by design): the row-block writer's mask byte stores, fused form, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-diag_c4m}
mkdir -p "$OUT"
LIBS=(abv/final.so abv/d_nomask.so)
for r in 1 2 3; do
  for i in 0 1; do
    MACM_LIB="$PWD/${LIBS[$i]}" timeout -k 10 200 python bench.py --no-cpu-baseline --env tdm --steps 20 --warmup 5 > "$OUT/c4_window_v${i}_r$r.json" 2> "$OUT/c4_window_v${i}_r$r.err" || exit $?
  done
done
echo ALLDONE
