#!/bin/bash
# Same-session A/B of library variants on the workgroup-path configs: tools/ab_c3.sh OUT lib1.so lib2.so ...
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
cfg c3_window 4 --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
cfg c3_bots 3 --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200 && \
cfg c5_window 3 --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
echo ALLDONE
