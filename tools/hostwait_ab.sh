#!/bin/bash
# A/B of the host's wait for the timed launch (bench.py --host-wait default / spin) at the driver's
# command, alternated 6 times in one session.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-hostwait}
mkdir -p "$OUT"
for r in 1 2 3 4 5 6; do
  for hw in default spin; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --host-wait $hw \
      > "$OUT/m_window_${hw}_r${r}.json" 2> "$OUT/m_window_${hw}_r${r}.err" || exit $?
  done
done
echo ALLDONE
