#!/bin/bash
# End-of-round evidence (round 5): every GPU test, the smoke, the PMC passes of the driver's command
# (M, trajectory outputs: the default form) and of the C4 window (the traffic bench.py quotes, keyed to
# this library's sha256), rocprofv3 kernel traces of the driver's command and of the C5 / C3 windows,
# the SQ counters of the workgroup kernels at C5 and C3, the driver's command itself and the M closed
# loop. Each step has its own time limit; a failing step ends the script.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-final_r05}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
st() { echo "$1 rc=$2" | tee -a "$R/$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1; st pytest_gpu $?
timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; st smoke $?
timeout -k 10 400 bash tools/pmc.sh "$OUT/pmc_m" --gpus 1 --steps 20 --warmup 5 > "$OUT/pmc_m.log" 2>&1; st pmc_m $?
timeout -k 10 400 bash tools/pmc.sh "$OUT/pmc_c4" --env tdm --steps 20 --warmup 5 > "$OUT/pmc_c4.log" 2>&1; st pmc_c4 $?
prof() {  # $1 = name, rest = bench args
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/rocprof_$name" -o $name -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/$OUT/rocprof_$name.json" 2> "$R/$OUT/rocprof_$name.err")
}
prof m --gpus 1 --steps 20 --warmup 5; st rocprof_m $?
prof c5 --envs 2048 --agents 1024 --steps 10 --warmup 2; st rocprof_c5 $?
prof c3 --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5; st rocprof_c3 $?
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
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/m_driver.json" 2> "$OUT/m_driver.err"; st m_driver $?
timeout -k 10 400 python bench.py --policy bots --steps 100 --warmup 300 --no-cpu-baseline > "$OUT/m_bots.json" 2> "$OUT/m_bots.err"; st m_bots $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
