#!/bin/bash
# Same-session A/B of library variants on the TDM configs: tools/ab_c4.sh OUT lib1.so lib2.so ...
# C4 window (6 alternations), C4 steady, the 512-env shard's window and steady state (3 each).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
LIBS=("$@")
cfg() {
  local name=$1 reps=$2; shift 2
  for r in $(seq 1 $reps); do
    for i in "${!LIBS[@]}"; do
      MACM_LIB="$PWD/${LIBS[$i]}" timeout -k 10 200 python bench.py --no-cpu-baseline "$@" \
        > "$OUT/${name}_v${i}_r${r}.json" 2> "$OUT/${name}_v${i}_r${r}.err" || return $?
    done
  done
  echo "$name done"
}
cfg c4_window 6 --env tdm --steps 20 --warmup 5 && \
cfg c4_steady 3 --env tdm --steps 1000 --warmup 100 && \
cfg c4_512_window 3 --env tdm --envs 512 --steps 20 --warmup 5 && \
cfg c4_512_steady 3 --env tdm --envs 512 --steps 1000 --warmup 100 && \
cfg c4_bots 3 --env tdm --policy bots --steps 100 --warmup 100 && \
echo ALLDONE
