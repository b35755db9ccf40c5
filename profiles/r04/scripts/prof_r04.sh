#!/bin/bash
# Round-4 per-kernel evidence for the level-step work: rocprofv3 kernel-trace stats of the C5 window,
# the M and C3 closed loops, and SQ PMC passes of the C5 window (kernel B = flock_solve_wg).
#   profiles/r04/scripts/prof_r04.sh OUTNAME [MACM_LIB path]
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${1:-prof_r04}"
mkdir -p "$OUT"
[ $# -ge 2 ] && export MACM_LIB="$R/$2"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
kt() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  st "$name" $?
}
pmc() {  # name, counters... (bench args from C5)
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc "$@" -d "$OUT/$name" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline $C5 > "$OUT/$name.json" 2> "$OUT/$name.err"
  st "$name" $?
}
C5="--envs 2048 --agents 1024 --steps 10 --warmup 2"
kt c5_window $C5
kt m_bots --policy bots --steps 100 --warmup 300
kt c3_bots --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200
pmc c5_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY
pmc c5_sq2 SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
echo ALLDONE | tee -a "$OUT/status.txt"
