#!/bin/bash
# Round-4 box session: confirmation of the knob-sweep candidates (sweep look-ahead 1, priority-2
# threshold 1, both), four alternating rounds (two A/B passes).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04kc}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
V=head,swa1,p2t1,sp
bash tools/ab_r04.sh "$(basename $OUT)/ab1" "mtr:$V mss:$V c4:$V c2:$V mbots:$V" > "$OUT/ab1.log" 2>&1; st ab1 $?
bash tools/ab_r04.sh "$(basename $OUT)/ab2" "mtr:$V mss:$V c4:$V c2:$V mbots:$V" > "$OUT/ab2.log" 2>&1; st ab2 $?
echo ALLDONE | tee -a "$OUT/status.txt"
