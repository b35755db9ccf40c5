#!/bin/bash
# Round-4 box session: level-step microbenchmark (chain-lane variants), the ADVICE-fix tests, the
# host-wait A/B and the HEAD phase profile.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04d}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 5 120 tools/build/ubench_level > "$OUT/ubench_level.txt" 2>&1; st ubench $?
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_tdm_wg.py tests/test_gpu_trajectory.py tests/test_gpu_tdm_spill.py tests/test_gpu_dense.py \
  > "$OUT/pytest.log" 2>&1; st pytest $?
for r in 1 2; do
  for hw in default spin; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-wait $hw \
      > "$OUT/m_${hw}_$r.json" 2> "$OUT/m_${hw}_$r.err"; st "bench_${hw}_$r" $?
  done
done
bash tools/gpu_r04c.sh "$(basename $OUT)/phases"; st phases $?
echo ALLDONE | tee -a "$OUT/status.txt"
