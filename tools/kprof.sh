#!/bin/bash
# Per-kernel rocprofv3 stats of library variants on one bench config, one box:
#   tools/kprof.sh OUTNAME lib1.so lib2.so ... [-- bench args]
# writes gpurun_out/OUTNAME/v<i>/run_kernel_stats.csv and summary.txt (avg us per kernel).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ $# -gt 0 ] && shift
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for i in "${!LIBS[@]}"; do
  export MACM_LIB="$R/${LIBS[$i]}"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/v$i" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/$OUT/v$i.json" 2> "$R/$OUT/v$i.err" || exit $?
done
cd "$R"
python3 tools/kprof_summary.py "$OUT" "${LIBS[@]}" | tee "$OUT/summary.txt"
echo ALLDONE
