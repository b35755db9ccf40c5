#!/bin/bash
# round 6: the split TDM observation — its equality tests, the TDM suites (which now run it by
# default below 2048 envs), then C4 timings of both forms at 512 and 4096 envs
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-split}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_tdm_split.py \
  tests/test_gpu_tdm.py tests/test_gpu_tdm_spill.py tests/test_gpu_tdm_wg.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -5 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?; echo "$name rc=$rc"; return $rc; }
MACM_TDM_SPLIT_OBS=1 run c4_512_split --env tdm --envs 512 --steps 20 --warmup 5 --no-cpu-baseline && \
MACM_TDM_SPLIT_OBS=0 run c4_512_fused --env tdm --envs 512 --steps 20 --warmup 5 --no-cpu-baseline && \
MACM_TDM_SPLIT_OBS=1 run c4_512_split_steady --env tdm --envs 512 --steps 1000 --warmup 100 --no-cpu-baseline && \
MACM_TDM_SPLIT_OBS=1 run c4_1024_split --env tdm --envs 1024 --steps 20 --warmup 5 --no-cpu-baseline && \
MACM_TDM_SPLIT_OBS=0 run c4_1024_fused --env tdm --envs 1024 --steps 20 --warmup 5 --no-cpu-baseline && \
MACM_TDM_SPLIT_OBS=1 run c4_2048_split --env tdm --envs 2048 --steps 20 --warmup 5 --no-cpu-baseline && \
MACM_TDM_SPLIT_OBS=0 run c4_2048_fused --env tdm --envs 2048 --steps 20 --warmup 5 --no-cpu-baseline && \
MACM_TDM_SPLIT_OBS=1 run c4_4096_split --env tdm --steps 20 --warmup 5 --no-cpu-baseline && \
MACM_TDM_SPLIT_OBS=0 run c4_4096_fused --env tdm --steps 20 --warmup 5 --no-cpu-baseline
