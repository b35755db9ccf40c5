#!/bin/bash
# Round-4 box session: parity tests of the kernel C / DFS / TDM-mask changes, the host-gap
# breakdown, then A/B of the library variants (ab/*.so) per workload.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04f}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_grid.py tests/test_gpu_fullsize.py tests/test_gpu_dense.py tests/test_gpu_parity.py \
  tests/test_gpu_tdm.py tests/test_gpu_tdm_spill.py > "$OUT/pytest.log" 2>&1; st pytest $?
timeout -k 10 120 python tools/host_gap.py > "$OUT/host_gap.json" 2>&1; st host_gap $?
timeout -k 10 120 python tools/host_gap.py --spin > "$OUT/host_gap_spin.json" 2>&1; st host_gap_spin $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c5r:prev,nc2,pr,pf,sl c3:prev,cells128 c4:pf,tm" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
