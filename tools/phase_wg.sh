#!/bin/bash
# Phase cycles of the split step's kernel C and solver (stamp builds ab/stamps_<variant>.so):
#   tools/phase_wg.sh OUTNAME variant ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for v in "$@"; do
 MACM_STAMPS_LIB=$PWD/ab/stamps_$v.so timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --warmup 5 --steps 10 --json $OUT/c3_$v.json > $OUT/c3_$v.log 2>&1 || exit $?
 MACM_STAMPS_LIB=$PWD/ab/stamps_$v.so timeout -k 10 200 python tools/phase_profile.py --envs 2048 --agents 1024 --warmup 2 --steps 4 --json $OUT/c5_$v.json > $OUT/c5_$v.log 2>&1 || exit $?
 MACM_STAMPS_LIB=$PWD/ab/stamps_$v.so timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --policy bots --warmup 200 --steps 10 --json $OUT/c3b_$v.json > $OUT/c3b_$v.log 2>&1 || exit $?
done
echo ALLDONE
