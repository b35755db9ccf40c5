#!/bin/bash
# Round-4 box session: rollout load balancing (order by launch index, >= 32 steps) + DFS and level-walk cost probes: parity + A/B.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04y}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_rollout.py tests/test_gpu_headline.py tests/test_gpu_bots.py \
  tests/test_gpu_tdm.py tests/test_gpu_wide_levels.py > "$OUT/pytest.log" 2>&1; st pytest $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "mtr:nobal,bal,dfs2x,lvl2x,dfslean mbots:nobal,bal,dfs2x,lvl2x,dfslean c4:bal,dfslean c4bots:nobal,bal,dfslean c3bots:nobal,bal" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
