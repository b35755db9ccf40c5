#!/bin/bash
# End-of-round check of the final tree: every GPU test, smoke, the driver's bench command.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-final7}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$R/$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1; st pytest_gpu $?
timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; st smoke $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/m_driver.json" 2> "$OUT/m_driver.err"; st m_driver $?
timeout -k 10 400 python bench.py > "$OUT/m_default.json" 2> "$OUT/m_default.err"; st m_default $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
