#!/bin/bash
# Build a variant of libmacm_hip.so with extra compile flags for A/B timing (tools/ab.sh):
#   tools/build_variant.sh NAME [-DFLAG ...]   ->  ab/NAME.so  (ab/ is git-ignored, ships with gpurun)
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p ab/build_$NAME
SRC="flock_step_w64 flock_rollout_w64 flock_step_wg tdm_step_wg bots env_reset actions_check macm_capi"
for f in $SRC; do
  X=""; [ $f = flock_rollout_w64 ] && X="-mllvm -disable-machine-licm"  # as the Makefile
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-result $X "$@" \
    -c -o ab/build_$NAME/$f.o gym-macm_amd/csrc/$f.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ab/$NAME.so ab/build_$NAME/*.o
rm -rf ab/build_$NAME
echo "built ab/$NAME.so"
