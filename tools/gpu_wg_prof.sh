#!/bin/bash
# Workgroup-path evidence: pytest -m gpu, smoke, then C3 / C5 benches and rocprofv3 kernel
# stats of the split kernels (C5 from reset and after a 100-step warm-up).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-wg}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/status.txt"; if [ $rc -ne 0 ] && [ "$name" != pytest_gpu -o $rc -ne 1 ]; then echo STOP | tee -a "$OUT/status.txt"; exit $rc; fi; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
step pytest_gpu timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
step smoke timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1
fi
step c3 timeout -k 10 300 python bench.py --envs 4096 --agents 256 --flocks 4 --steps 60 --warmup 5 > "$OUT/c3.json" 2> "$OUT/c3.err"
step c5 timeout -k 10 300 python bench.py --envs 2048 --agents 1024 --steps 6 --warmup 2 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err"
cd /tmp && export TMPDIR=/tmp
step prof_c3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c3" -o run -- \
  python3 "$R/bench.py" --envs 4096 --agents 256 --flocks 4 --steps 40 --warmup 5 --no-cpu-baseline > "$R/$OUT/prof_c3.json" 2> "$R/$OUT/prof_c3.err"
step prof_c5 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_c5" -o run -- \
  python3 "$R/bench.py" --envs 2048 --agents 1024 --steps 6 --warmup 2 --no-cpu-baseline > "$R/$OUT/prof_c5.json" 2> "$R/$OUT/prof_c5.err"
cd "$R"
if [ "${C5_WARM:-1}" = 1 ]; then
step c5_warm timeout -k 10 600 python bench.py --envs 2048 --agents 1024 --steps 10 --warmup 100 --no-cpu-baseline > "$OUT/c5_warm.json" 2> "$OUT/c5_warm.err"
fi
echo ALLDONE | tee -a "$OUT/status.txt"
