#!/bin/bash
# Round 6: only the last S steps of a full-chip TDM rollout observed in the tail (MACM_TDM_TAIL_STEPS),
# fused vs S = 2 / 4 / 7 at 4096 envs and S = 5 at 2048, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-tail_ab5}
mkdir -p "$OUT"
run() {
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
F="MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0"
T="MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1"
for r in 1 2 3; do
  run "c4_window_v0_r$r" "$F" --env tdm --steps 20 --warmup 5 || exit $?
  for st in 2 4 7; do
    run "c4_window_vs${st}_r$r" "$T MACM_TDM_TAIL_STEPS=$st" --env tdm --steps 20 --warmup 5 || exit $?
  done
  run "e2048_window_v0_r$r" "$F" --env tdm --envs 2048 --steps 20 --warmup 5 || exit $?
  run "e2048_window_vs5_r$r" "$T MACM_TDM_TAIL_STEPS=5" --env tdm --envs 2048 --steps 20 --warmup 5 || exit $?
  run "c4_steady_v0_r$r" "$F" --env tdm --steps 1000 --warmup 100 || exit $?
  run "c4_steady_vs100_r$r" "$T MACM_TDM_TAIL_STEPS=100" --env tdm --steps 1000 --warmup 100 || exit $?
  echo "round $r done"
done
echo ALLDONE
