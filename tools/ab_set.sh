#!/bin/bash
# A/B timing of library variants over a set of workloads in one GPU session, alternating variants
# (fresh process each) twice so clock drift hits all alike:
#   tools/ab_set.sh OUTNAME "mtr mss mbots c3 c4 c5" lib1.so lib2.so ...
# Summary: python tools/ab_set_summary.py gpurun_out/OUTNAME
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; WL=$2; shift 2
mkdir -p "$OUT"
args() {
  case $1 in
    mtr) echo "--steps 20 --warmup 5" ;;                       # the driver's window
    mss) echo "--steps 1000 --warmup 100" ;;
    mbots) echo "--policy bots --steps 100 --warmup 300" ;;
    c2) echo "--envs 1024 --steps 1000 --warmup 100" ;;
    c3) echo "--agents 256 --flocks 4 --steps 20 --warmup 5" ;;
    c3bots) echo "--agents 256 --flocks 4 --policy bots --steps 50 --warmup 250" ;;
    t128) echo "--env tdm --teams 64,64 --envs 1024 --steps 20 --warmup 5" ;;
    t512) echo "--env tdm --teams 256,256 --envs 256 --steps 5 --warmup 2" ;;
    c3ss) echo "--agents 256 --flocks 4 --steps 100 --warmup 50" ;;
    c4) echo "--env tdm --steps 20 --warmup 5" ;;
    c4bots) echo "--env tdm --policy bots --steps 100 --warmup 100" ;;
    c5) echo "--envs 2048 --agents 1024 --steps 10 --warmup 2 --launch step" ;;
    c5r) echo "--envs 2048 --agents 1024 --steps 10 --warmup 2" ;;            # rollout form (driver)
  esac
}
for r in 1 2; do
  for w in $WL; do
    i=0
    for lib in "$@"; do
      # shellcheck disable=SC2046
      MACM_LIB="$PWD/$lib" timeout -k 10 150 python bench.py --no-cpu-baseline $(args "$w") \
        > "$OUT/${w}_v${i}_r${r}.json" 2> "$OUT/${w}_v${i}_r${r}.err" || exit $?
      i=$((i + 1))
    done
  done
done
echo ALLDONE
