#!/bin/bash
# Build a variant of libmacm_hip.so with extra compile flags for A/B timing (tools/ab.sh):
#   tools/build_variant.sh NAME [-DFLAG ...]   ->  abv/NAME.so  (abv/ is git-ignored and ships with gpurun;
#   ab/ holds old variants and does not ship: .gpurunignore)
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p abv/build_$NAME
PIDS=()
SRC="flock_step_w64 flock_rollout_w64 flock_step_wg flock_big tdm_step_wg bots env_reset actions_check macm_capi"
for f in $SRC; do
  X=""; [ $f = flock_rollout_w64 ] && X="-mllvm -disable-machine-licm"  # as the Makefile
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-result $X "$@" \
    -c -o abv/build_$NAME/$f.o gym-macm_amd/csrc/$f.hip &
  PIDS+=($!)
done
for p in "${PIDS[@]}"; do wait "$p" || { echo "compile failed: abv/$NAME.so not built" >&2; rm -rf abv/build_$NAME; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o abv/$NAME.so abv/build_$NAME/*.o
rm -rf abv/build_$NAME
echo "built abv/$NAME.so"
