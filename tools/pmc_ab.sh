#!/bin/bash
# SQ instruction counters per kernel for library variants: tools/pmc_ab.sh OUT lib1 lib2 ... -- bench args
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$R/gpurun_out/$1; shift
mkdir -p "$OUT"
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ $# -gt 0 ] && shift
cd /tmp && export TMPDIR=/tmp
for i in "${!LIBS[@]}"; do
  export MACM_LIB="$R/${LIBS[$i]}"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY \
    -d "$OUT/v$i" -o run -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/v$i.json" 2> "$OUT/v$i.err" || exit $?
done
cd "$R"
python3 tools/pmc_ab_summary.py "$OUT" "${LIBS[@]}" | tee "$OUT/summary.txt"
echo ALLDONE
