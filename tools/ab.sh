#!/bin/bash
# A/B timing of library variants in one GPU session: tools/ab.sh OUTNAME lib1.so lib2.so ... [-- bench args]
# Alternates the variants 3 times (fresh process each) so clock/thermal drift hits all alike.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ $# -gt 0 ] && shift
for r in 1 2 3; do
  for i in "${!LIBS[@]}"; do
    MACM_LIB="$PWD/${LIBS[$i]}" timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline "$@" \
      > "$OUT/v${i}_r${r}.json" 2> "$OUT/v${i}_r${r}.err" || exit $?
  done
done
echo ALLDONE
