#!/bin/bash
# Round 6: the TDM tail observation against the fused and split forms, one session, alternated 3 times.
# tools/tail_ab.sh OUT
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-tail_ab}
mkdir -p "$OUT"
run() {  # name, env assignments (space separated), bench args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
for r in 1 2 3; do
  run "c4_window_v0_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0" --env tdm --steps 20 --warmup 5 || exit $?
  run "c4_window_v1_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1" --env tdm --steps 20 --warmup 5 || exit $?
  run "c4_steady_v0_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0" --env tdm --steps 1000 --warmup 100 || exit $?
  run "c4_steady_v1_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1" --env tdm --steps 1000 --warmup 100 || exit $?
  run "c4_2048_window_v0_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0" --env tdm --envs 2048 --steps 20 --warmup 5 || exit $?
  run "c4_2048_window_v1_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1" --env tdm --envs 2048 --steps 20 --warmup 5 || exit $?
  for w in 0 512 1536; do
    run "c4_512_window_v1w${w}_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1 MACM_TDM_TAIL_WORKERS=$w" --env tdm --envs 512 --steps 20 --warmup 5 || exit $?
  done
  run "c4_512_window_v0_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0" --env tdm --envs 512 --steps 20 --warmup 5 || exit $?
  run "c4_512_window_vs_r$r" "MACM_TDM_SPLIT_OBS=1 MACM_TDM_TAIL_OBS=0" --env tdm --envs 512 --steps 20 --warmup 5 || exit $?
  run "c4_512_steady_v0_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=0" --env tdm --envs 512 --steps 1000 --warmup 100 || exit $?
  run "c4_512_steady_vs_r$r" "MACM_TDM_SPLIT_OBS=1 MACM_TDM_TAIL_OBS=0" --env tdm --envs 512 --steps 1000 --warmup 100 || exit $?
  run "c4_512_steady_v1_r$r" "MACM_TDM_SPLIT_OBS=0 MACM_TDM_TAIL_OBS=1" --env tdm --envs 512 --steps 1000 --warmup 100 || exit $?
  echo "round $r done"
done
echo ALLDONE
