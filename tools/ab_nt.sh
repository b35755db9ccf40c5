#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ntc4; mkdir -p $OUT
for r in 1 2 3; do for v in base ntout ntall; do
  MACM_LIB=$PWD/ab/$v.so timeout -k 10 120 python bench.py --env tdm --steps 300 --warmup 30 --no-cpu-baseline > $OUT/${v}_r${r}_c4.json 2>/dev/null || exit $?
  MACM_LIB=$PWD/ab/$v.so timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/${v}_r${r}_mss.json 2>/dev/null || exit $?
  MACM_LIB=$PWD/ab/$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${v}_r${r}_mtr.json 2>/dev/null || exit $?
done; done
echo ALLDONE
