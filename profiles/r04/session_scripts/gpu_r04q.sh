#!/bin/bash
# Round-4 box session: the whole GPU suite on the candidate library (kernel B shared dummy, serial
# walk prefetch, wide-level slot ranges), A/B against the last commit.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04q}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1; st pytest_gpu $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "mbots:head,fin1 c3bots:head,fin1 c5r:head,fin1 c3:head,fin1 mtr:head,fin1 c4:head,fin1" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
