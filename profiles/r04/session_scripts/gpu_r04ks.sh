#!/bin/bash
# Round-4 box session: re-sweep of the wave kernel's compile-time thresholds at HEAD (timing only;
# a winner gets the whole GPU suite before it is kept).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04ks}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
V=head,lmi2,lmi8,rec6,rec3,swa3,swa1,p2t1,p2t8
bash tools/ab_r04.sh "$(basename $OUT)/ab" "mtr:$V mss:$V c4:$V mbots:head,lmi2,lmi8,rec6,rec3,p2t1,p2t8" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
