#!/bin/bash
# A/B of library variants per workload in one session, alternating (fresh process each), 2 rounds:
#   tools/ab_r04.sh OUTNAME "wl:lib1,lib2 wl2:lib1,lib3 ..."   (libs are ab/<name>.so)
# Workload names as tools/ab_set.sh. Summary: python tools/ab_set_summary.py gpurun_out/OUTNAME
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; SPEC=$2
mkdir -p "$OUT"
args() {
  case $1 in
    mtr) echo "--steps 20 --warmup 5" ;;
    mstep) echo "--launch step --steps 20 --warmup 5" ;;
    mss) echo "--steps 1000 --warmup 100" ;;
    mbots) echo "--policy bots --steps 100 --warmup 300" ;;
    c2) echo "--envs 1024 --steps 1000 --warmup 100" ;;
    c3) echo "--agents 256 --flocks 4 --steps 20 --warmup 5" ;;
    c3bots) echo "--agents 256 --flocks 4 --policy bots --steps 50 --warmup 250" ;;
    c4) echo "--env tdm --steps 20 --warmup 5" ;;
    c4bots) echo "--env tdm --policy bots --steps 100 --warmup 100" ;;
    c5r) echo "--envs 2048 --agents 1024 --steps 10 --warmup 2" ;;
  esac
}
for r in 1 2; do
  for item in $SPEC; do
    w=${item%%:*}; libs=${item#*:}
    for lib in ${libs//,/ }; do
      # shellcheck disable=SC2046
      MACM_LIB="$PWD/ab/$lib.so" timeout -k 10 150 python bench.py --no-cpu-baseline $(args "$w") \
        > "$OUT/${w}_${lib}_r${r}.json" 2> "$OUT/${w}_${lib}_r${r}.err" || exit $?
      python3 -c "import json,sys; j=json.load(open('$OUT/${w}_${lib}_r${r}.json')); print('$w $lib r$r', round(j['ms_per_step']*1e3,2), 'us/step', round(j['roofline']['kernel_ms']*1e3,2))"
    done
  done
done
echo ALLDONE
