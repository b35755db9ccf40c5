#!/bin/bash
# Round-4 box session: the whole GPU suite on the current library, the C4 mask-staging PMC (HBM
# bytes, pair tiles vs staged mask), the host gap in bench.py's call sequence, and A/B timings.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04g}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1; st pytest_gpu $?
for v in pf tm; do
  MACM_LIB="$R/ab/$v.so" timeout -k 10 300 bash tools/pmc.sh "$OUT/pmc_c4_$v" --env tdm --steps 20 --warmup 5 \
    > "$OUT/pmc_c4_$v.log" 2>&1; st "pmc_c4_$v" $?
done
timeout -k 10 120 python tools/host_gap.py --bench-like > "$OUT/host_gap_bench_like.json" 2>&1; st host_gap_bl $?
timeout -k 10 120 python tools/host_gap.py > "$OUT/host_gap.json" 2>&1; st host_gap $?
bash tools/ab_r04.sh "$(basename $OUT)/ab" "c5r:pr,cur c3:prev,cur c3bots:prev,cur mbots:prev,cur" > "$OUT/ab.log" 2>&1; st ab $?
echo ALLDONE | tee -a "$OUT/status.txt"
