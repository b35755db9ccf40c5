#!/bin/bash
# End-of-round evidence (round 4): every GPU test, smoke, the driver's bench command and the default
# bench, rocprofv3 kernel-trace stats of the driver's command, the PMC passes of the driver's command
# (M) and of the TDM C4 window (the traffic bench.py quotes, keyed to this library's sha256), and
# every config's bench line. Each step has its own time limit; a failing step ends the script.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-final_r04}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$R/$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1; st pytest_gpu $?
timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; st smoke $?
timeout -k 10 400 bash tools/pmc.sh "$OUT/pmc_m" --gpus 1 --steps 20 --warmup 5 > "$OUT/pmc_m.log" 2>&1; st pmc_m $?
timeout -k 10 400 bash tools/pmc.sh "$OUT/pmc_c4" --env tdm --steps 20 --warmup 5 > "$OUT/pmc_c4.log" 2>&1; st pmc_c4 $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/rocprof" -o m -- \
  python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$R/$OUT/m_rocprof_bench.json" 2> "$R/$OUT/m_rocprof.err"); st rocprof $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/m_driver.json" 2> "$OUT/m_driver.err"; st m_driver $?
timeout -k 10 400 python bench.py > "$OUT/m_default.json" 2> "$OUT/m_default.err"; st m_default $?
timeout -k 10 400 python bench.py --policy bots --steps 100 --warmup 300 --no-cpu-baseline > "$OUT/m_bots.json" 2> "$OUT/m_bots.err"; st m_bots $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
