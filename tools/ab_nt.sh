#!/bin/bash
# Round 6: nontemporal obs stores in the row-block writer, A/B at C4 (4096, 512 fused and tail), 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ab_nt}
mkdir -p "$OUT"
LIBS=("${@:2}")
for r in 1 2 3; do
  for i in "${!LIBS[@]}"; do
    L="$PWD/${LIBS[$i]}"
    MACM_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --env tdm --steps 20 --warmup 5 > "$OUT/c4_window_v${i}_r$r.json" 2> "$OUT/c4_window_v${i}_r$r.err" || exit $?
    MACM_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --env tdm --steps 1000 --warmup 100 > "$OUT/c4_steady_v${i}_r$r.json" 2> "$OUT/c4_steady_v${i}_r$r.err" || exit $?
    MACM_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --env tdm --envs 512 --steps 20 --warmup 5 > "$OUT/c4_512_window_v${i}_r$r.json" 2> "$OUT/c4_512_window_v${i}_r$r.err" || exit $?
    MACM_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --env tdm --policy bots --steps 100 --warmup 100 > "$OUT/c4_bots_v${i}_r$r.json" 2> "$OUT/c4_bots_v${i}_r$r.err" || exit $?
  done
done
echo ALLDONE
