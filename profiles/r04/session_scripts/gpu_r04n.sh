#!/bin/bash
# Round-4 box session: level-step microbenchmark (shared dummy slot variants), M-bots phase cycles
# at HEAD (level-ordered wide slots).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04n}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 300 tools/build/ubench_level > "$OUT/ubench_level.txt" 2>&1; st ubench $?
S="$R/ab/stamps_head.so"
MACM_STAMPS_LIB=$S timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 64 --policy bots --warmup 300 --steps 10 --json $OUT/mbots.json > $OUT/mbots.log 2>&1; st mbots $?
echo ALLDONE | tee -a "$OUT/status.txt"
