#!/bin/bash
# Round-4 box session: the whole GPU suite on the candidate library (pipelined strip-cell
# candidates, DFS record batch 8, DPP block scans), then A/B against the last committed forms.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04k}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1; st pytest_gpu $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c5r:ring,cand c3:ring,cand c3bots:ring,cand mtr:walk,cand mbots:walk,cand c4:walk,cand" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
