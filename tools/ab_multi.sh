#!/bin/bash
# Same-session A/B of library variants over several configs: tools/ab_multi.sh OUT lib1.so lib2.so
# Each config alternates the variants 3 times (fresh process each).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
LIBS=("$@")
cfg() {
  local name=$1; shift
  for r in 1 2 3; do
    for i in "${!LIBS[@]}"; do
      MACM_LIB="$PWD/${LIBS[$i]}" timeout -k 10 200 python bench.py --no-cpu-baseline "$@" \
        > "$OUT/${name}_v${i}_r${r}.json" 2> "$OUT/${name}_v${i}_r${r}.err" || return $?
    done
  done
  echo "$name done"
}
cfg m_window --steps 20 --warmup 5 && \
cfg m_steady --steps 1000 --warmup 100 && \
cfg m_bots --policy bots --steps 100 --warmup 300 && \
cfg c4_window --env tdm --steps 20 --warmup 5 && \
cfg c3_window --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
cfg c5_window --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
echo ALLDONE
