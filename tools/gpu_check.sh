#!/bin/bash
# One box session: the GPU suite, the smoke, the driver's bench command (default outputs form) and
# optional extra steps. Every step has its own time limit; a failing step ends the script.
#   tools/gpu_check.sh OUTNAME [extra...]    extra: overwrite | ubench | c5 | c3 | mbots | c4
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-check}
shift
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
st() { echo "$1 rc=$2" | tee -a "$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1; st pytest $?
timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; st smoke $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/m_driver.json" 2> "$OUT/m_driver.err"; st m_driver $?
for x in "$@"; do
  case $x in
    overwrite) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --outputs overwrite --no-cpu-baseline > "$OUT/m_overwrite.json" 2> "$OUT/m_overwrite.err"; st overwrite $? ;;
    ubench) timeout -k 10 300 tools/build/ubench_level > "$OUT/ubench_level.txt" 2>&1; st ubench $? ;;
    c5) timeout -k 10 300 python bench.py --envs 2048 --agents 1024 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err"; st c5 $? ;;
    c3) timeout -k 10 300 python bench.py --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err"; st c3 $? ;;
    mbots) timeout -k 10 300 python bench.py --policy bots --steps 100 --warmup 300 --no-cpu-baseline > "$OUT/m_bots.json" 2> "$OUT/m_bots.err"; st mbots $? ;;
    c4) timeout -k 10 300 python bench.py --env tdm --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c4.json" 2> "$OUT/c4.err"; st c4 $? ;;
  esac
done
echo ALLDONE | tee -a "$OUT/status.txt"
