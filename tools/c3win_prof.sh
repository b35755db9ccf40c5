#!/bin/bash
# Phase shares of the workgroup path in the C3 window (random actions, steps 6-15 from reset) and
# bench lines of TDM above 64 agents (the workgroup TDM step).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-c3win}; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
MACM_STAMPS_LIB=$PWD/ab/stamps_head.so timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --warmup 5 --steps 10 --json $OUT/c3w.json > $OUT/c3w.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --env tdm --teams 64,64 --envs 1024 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/tdm_64x2.json 2> $OUT/tdm_64x2.err || exit $?
timeout -k 10 200 python bench.py --env tdm --teams 256,256 --envs 256 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/tdm_256x2.json 2> $OUT/tdm_256x2.err || exit $?
echo ALLDONE
