#!/bin/bash
# PMC passes for the bench workload (counters in their own runs, kernel-trace only).
# usage: tools/pmc.sh OUTDIR [bench args...]
set -u
OUT=$1; shift
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$REPO/$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc "$@" -d "$REPO/$OUT/pmc_$name" -o run -- \
    python3 "$REPO/bench.py" --no-cpu-baseline "${BENCH_ARGS[@]}" > "$REPO/$OUT/pmc_$name.json" 2> "$REPO/$OUT/pmc_$name.err"
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
BENCH_ARGS=("$@")
# the library these passes measure (tools/pmc_summary.py records it; bench.py checks it)
sha256sum "${MACM_LIB:-$REPO/gym-macm_amd/libmacm_hip.so}" > "$REPO/$OUT/lib.sha256"
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY && \
run sq2 SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT GRBM_GUI_ACTIVE
