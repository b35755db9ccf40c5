#!/bin/bash
# Round 6: the tail observation after the load-before-claim change, fused vs tail, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-tail_ab4}
mkdir -p "$OUT"
run() {
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
F="MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0"
T="MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1"
for r in 1 2 3; do
  for E in 512 1024 2048; do
    run "e${E}_window_v0_r$r" "$F" --env tdm --envs $E --steps 20 --warmup 5 || exit $?
    run "e${E}_window_v1_r$r" "$T" --env tdm --envs $E --steps 20 --warmup 5 || exit $?
  done
  run "e512_steady_v0_r$r" "$F" --env tdm --envs 512 --steps 1000 --warmup 100 || exit $?
  run "e512_steady_v1_r$r" "$T" --env tdm --envs 512 --steps 1000 --warmup 100 || exit $?
  run "c4_window_v0_r$r" "$F" --env tdm --steps 20 --warmup 5 || exit $?
  run "c4_window_vh256_r$r" "$T MACM_TDM_TAIL_HEAVY=256" --env tdm --steps 20 --warmup 5 || exit $?
  run "c4_window_vh4096_r$r" "$T MACM_TDM_TAIL_HEAVY=4096" --env tdm --steps 20 --warmup 5 || exit $?
  echo "round $r done"
done
echo ALLDONE
