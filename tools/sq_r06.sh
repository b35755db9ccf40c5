#!/bin/bash
# Round 6: the per-kernel SQ counters of the workgroup kernels at C5 and C3 at the final library (kernel
# B's wait / VALU ratio), two passes each (counter limits per pass); summarise with
# tools/sq_kernel_summary.py. Each pass has its own time limit; a failing pass ends the script.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-sq_r06}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
st() { echo "$1 rc=$2" | tee -a "$R/$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
sqpass() {  # $1 = name, $2 = counters, rest = bench args
  local name=$1 ctrs=$2; shift 2
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $ctrs -d "$R/$OUT/sq_$name" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/$OUT/sq_$name.json" 2> "$R/$OUT/sq_$name.err")
}
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY"
SQ2="SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VALU GRBM_GUI_ACTIVE"
sqpass c5_1 "$SQ1" --envs 2048 --agents 1024 --steps 10 --warmup 2; st sq_c5_1 $?
sqpass c5_2 "$SQ2" --envs 2048 --agents 1024 --steps 10 --warmup 2; st sq_c5_2 $?
sqpass c3_1 "$SQ1" --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5; st sq_c3_1 $?
sqpass c3_2 "$SQ2" --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5; st sq_c3_2 $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
