#!/bin/bash
# End-of-round evidence (round 3): every GPU test, smoke, the driver's bench command, its rocprofv3
# kernel-trace stats and the PMC passes of the same command. Each step has its own time limit and a
# failing step ends the script.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-final_r03}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$R/$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1; st pytest_gpu $?
timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; st smoke $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/m_driver.json" 2> "$OUT/m_driver.err"; st m_driver $?
timeout -k 10 400 python bench.py > "$OUT/m_default.json" 2> "$OUT/m_default.err"; st m_default $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/rocprof" -o m -- \
  python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$R/$OUT/m_rocprof_bench.json" 2> "$R/$OUT/m_rocprof.err"); st rocprof $?
timeout -k 10 400 bash tools/pmc.sh "$OUT/pmc_m" --gpus 1 --steps 20 --warmup 5 > "$OUT/pmc.log" 2>&1; st pmc $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
