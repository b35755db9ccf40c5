#!/bin/bash
# Same-session A/B of library variants at the metric config (driver window and steady state) and C4:
# tools/ab_m.sh OUT lib1.so lib2.so ... ; the window alternates the variants 6 times, the others 3.
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
cfg m_window 6 --steps 20 --warmup 5 && \
cfg m_steady 3 --steps 1000 --warmup 100 && \
cfg c4_window 3 --env tdm --steps 20 --warmup 5 && \
echo ALLDONE
