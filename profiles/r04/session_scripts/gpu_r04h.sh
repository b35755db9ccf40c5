#!/bin/bash
# Round-4 box session: parity of the flagged DFS walk and the fused DPP prefix maximum, the bench's
# host gap (first window vs repeated, events pre-recorded), A/B timings, phase stamps.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04h}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_dense.py tests/test_gpu_islands.py \
  tests/test_gpu_grid.py tests/test_gpu_wide_levels.py > "$OUT/pytest.log" 2>&1; st pytest $?
timeout -k 10 120 python tools/host_gap.py > "$OUT/host_gap.json" 2>&1; st host_gap $?
timeout -k 10 120 python tools/host_gap.py --prerecord > "$OUT/host_gap_pre.json" 2>&1; st host_gap_pre $?
for i in 1 2; do
  timeout -k 10 150 python bench.py --no-cpu-baseline > "$OUT/m_$i.json" 2> "$OUT/m_$i.err"; st "bench_m_$i" $?
done
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c5r:cur,dfs,nodpp c3bots:prev,dfs,walk,walk0,c512 c3:dfs,walk,c512" > "$OUT/ab.log" 2>&1; st ab $?
bash tools/phase_wg.sh "$(basename $OUT)/phase" dfs walk c512 > "$OUT/phase.log" 2>&1; st phase $?
echo ALLDONE | tee -a "$OUT/status.txt"
