#!/bin/bash
# Round 6: the tail observation's heavy-env form at 4096 and 2048 envs against the fused form, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-tail_ab3}
mkdir -p "$OUT"
run() {
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
F="MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0"
T="MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1"
for r in 1 2 3; do
  run "c4_window_v0_r$r" "$F" --env tdm --steps 20 --warmup 5 || exit $?
  for h in 128 256 512 1024; do
    run "c4_window_vh${h}_r$r" "$T MACM_TDM_TAIL_HEAVY=$h" --env tdm --steps 20 --warmup 5 || exit $?
  done
  run "c4_steady_v0_r$r" "$F" --env tdm --steps 1000 --warmup 100 || exit $?
  run "c4_steady_vh512_r$r" "$T MACM_TDM_TAIL_HEAVY=512" --env tdm --steps 1000 --warmup 100 || exit $?
  run "e2048_window_v0_r$r" "$F" --env tdm --envs 2048 --steps 20 --warmup 5 || exit $?
  run "e2048_window_vh256_r$r" "$T MACM_TDM_TAIL_HEAVY=256" --env tdm --envs 2048 --steps 20 --warmup 5 || exit $?
  run "e2048_window_vh2048_r$r" "$T" --env tdm --envs 2048 --steps 20 --warmup 5 || exit $?
  echo "round $r done"
done
echo ALLDONE
