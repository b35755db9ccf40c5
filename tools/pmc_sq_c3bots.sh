#!/bin/bash
# SQ counters of the workgroup path's kernels in the C3 closed loop (one pass per counter group).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pmc_c3bots}
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
A="--agents 256 --flocks 4 --policy bots --steps 20 --warmup 250 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY -d "$R/$OUT/sq" -o run -- python3 "$R/bench.py" $A > "$R/$OUT/sq.json" 2> "$R/$OUT/sq.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VALU GRBM_GUI_ACTIVE -d "$R/$OUT/sq2" -o run -- python3 "$R/bench.py" $A > "$R/$OUT/sq2.json" 2> "$R/$OUT/sq2.err" || exit $?
echo ALLDONE
