#!/bin/bash
# Round-4 box session: per-kernel traces and SQ PMC at HEAD (profiles/r04/scripts/prof_r04.sh), phase cycles of the
# closed loops and windows (stamp build of HEAD: ab/stamps_cand.so).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04l}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
bash profiles/r04/scripts/prof_r04.sh "$(basename $OUT)/prof" > "$OUT/prof.log" 2>&1; st prof $?
cd "$R"
S="$R/ab/stamps_cand.so"
MACM_STAMPS_LIB=$S timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 64 --policy bots --warmup 300 --steps 10 --json $OUT/mbots.json > $OUT/mbots.log 2>&1; st mbots $?
MACM_STAMPS_LIB=$S timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 64 --warmup 5 --steps 20 --json $OUT/mwin.json > $OUT/mwin.log 2>&1; st mwin $?
MACM_STAMPS_LIB=$S timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --policy bots --warmup 200 --steps 10 --json $OUT/c3b.json > $OUT/c3b.log 2>&1; st c3b $?
MACM_STAMPS_LIB=$S timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --warmup 5 --steps 10 --json $OUT/c3.json > $OUT/c3.log 2>&1; st c3 $?
echo ALLDONE | tee -a "$OUT/status.txt"
