#!/bin/bash
# Final tree check: GPU tests, smoke, the driver's bench command, workgroup-path lines (rollout form).
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-final6}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
st() { echo "$1 rc=$2" | tee -a "$R/$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1; st pytest_gpu $?
timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; st smoke $?
b() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; st "$name" $?; }
b m_driver --gpus 1 --steps 20 --warmup 5
b c3_driver --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5
b c3_steady --envs 4096 --agents 256 --flocks 4 --steps 100 --warmup 50 --no-cpu-baseline
b c5_driver --envs 2048 --agents 1024 --steps 20 --warmup 5
b c5_warm100 --envs 2048 --agents 1024 --steps 10 --warmup 100 --no-cpu-baseline
b c4_bots --env tdm --policy bots --steps 300 --warmup 30 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c3" -o run -- python3 "$R/bench.py" --no-cpu-baseline --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 > "$R/$OUT/prof_c3.json" 2> "$R/$OUT/prof_c3.err"; st prof_c3 $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
