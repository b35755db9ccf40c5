#!/bin/bash
# Round 6: where the tail observation stops paying (envs per launch), fused / split / tail, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-tail_ab2}
mkdir -p "$OUT"
run() {
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
for r in 1 2 3; do
  for E in 768 1024 1536; do
    run "e${E}_window_v0_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0" --env tdm --envs $E --steps 20 --warmup 5 || exit $?
    run "e${E}_window_vs_r$r" "MACM_TDM_SPLIT_OBS=1 MACM_TDM_TAIL_OBS=0" --env tdm --envs $E --steps 20 --warmup 5 || exit $?
    run "e${E}_window_v1_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1" --env tdm --envs $E --steps 20 --warmup 5 || exit $?
    run "e${E}_steady_v0_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0" --env tdm --envs $E --steps 500 --warmup 100 || exit $?
    run "e${E}_steady_v1_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1" --env tdm --envs $E --steps 500 --warmup 100 || exit $?
  done
  run "e512_window_v1w256_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1 MACM_TDM_TAIL_WORKERS=256" --env tdm --envs 512 --steps 20 --warmup 5 || exit $?
  run "e512_window_v1w1024_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1 MACM_TDM_TAIL_WORKERS=1024" --env tdm --envs 512 --steps 20 --warmup 5 || exit $?
  run "e512_window_v1_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1" --env tdm --envs 512 --steps 20 --warmup 5 || exit $?
  echo "round $r done"
done
echo ALLDONE
