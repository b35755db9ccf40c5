#!/bin/bash
# A/B timing of environment settings in one GPU session:
#   tools/ab_env.sh OUTNAME 'VAR=a' 'VAR=b' ... [-- bench args]
# Alternates the settings 3 times (fresh process each), like tools/ab.sh does for libraries.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
ENVS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
[ $# -gt 0 ] && shift
for r in 1 2 3; do
  for i in "${!ENVS[@]}"; do
    env ${ENVS[$i]} timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline "$@" \
      > "$OUT/v${i}_r${r}.json" 2> "$OUT/v${i}_r${r}.err" || exit $?
  done
done
echo ALLDONE
