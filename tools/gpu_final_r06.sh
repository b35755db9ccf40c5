#!/bin/bash
# End-of-round evidence (round 6): every GPU test, the smoke, the PMC passes of the driver's command (M,
# trajectory outputs) and of the C4 window (the traffic bench.py quotes, keyed to this library's
# sha256), rocprofv3 kernel traces (with --stats) of the driver's command and of the C5 / C3 / C4-shard
# windows, the driver's command itself. Each step has its own time limit; a failing step ends it.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-final_r06}
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
prof c4 --env tdm --steps 20 --warmup 5; st rocprof_c4 $?
prof c4_512 --env tdm --envs 512 --steps 20 --warmup 5; st rocprof_c4_512 $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/m_driver.json" 2> "$OUT/m_driver.err"; st m_driver $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
