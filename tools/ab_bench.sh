#!/bin/bash
# A/B of two bench.py versions (host-side timing changes) at the driver's command, alternated 8 times:
# tools/ab_bench.sh OUT old_bench.py new_bench.py
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for r in 1 2 3 4 5 6 7 8; do
  i=0
  for b in "$@"; do
    timeout -k 10 200 python "$b" --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/m_window_v${i}_r${r}.json" 2> "$OUT/m_window_v${i}_r${r}.err" || exit $?
    i=$((i + 1))
  done
done
echo ALLDONE
