#!/bin/bash
# A/B of HIP runtime environment settings at the driver's command (launch latency), alternated 6 times.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-hip_env_ab}
mkdir -p "$OUT"
for r in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/m_window_v0_r$r.json" 2> "$OUT/m_window_v0_r$r.err" || exit $?
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/m_window_vdev1_r$r.json" 2> "$OUT/m_window_vdev1_r$r.err" || exit $?
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/m_window_vdev0_r$r.json" 2> "$OUT/m_window_vdev0_r$r.err" || exit $?
done
echo ALLDONE
