#!/bin/bash
# Round-4 phase profile at HEAD (stamp build ab/stamps_head.so): C5 window (kernels A, DFS, B, C
# phase cycles), C3 window, the M closed loop (wave kernel).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04c}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
export MACM_STAMPS_LIB=$PWD/ab/stamps_head.so
timeout -k 10 200 python tools/phase_profile.py --envs 2048 --agents 1024 --warmup 2 --steps 4 --json $OUT/c5.json > $OUT/c5.log 2>&1; st c5 $?
timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --warmup 5 --steps 10 --json $OUT/c3.json > $OUT/c3.log 2>&1; st c3 $?
timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 64 --policy bots --warmup 300 --steps 10 --json $OUT/mbots.json > $OUT/mbots.log 2>&1; st mbots $?
timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 64 --warmup 5 --steps 20 --json $OUT/mwin.json > $OUT/mwin.log 2>&1; st mwin $?
echo ALLDONE | tee -a "$OUT/status.txt"
