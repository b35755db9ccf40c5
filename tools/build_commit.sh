#!/bin/bash
# Build libmacm_hip.so from the sources of a git commit, for A/B timing against the working tree:
#   tools/build_commit.sh NAME COMMIT [-DFLAG ...]  ->  ab/NAME.so  (ab/ is git-ignored, ships with gpurun)
set -eu
cd "$(dirname "$0")/.."
NAME=$1; COMMIT=$2; shift 2
D=ab/src_$NAME
rm -rf "$D" && mkdir -p "$D"
git archive "$COMMIT" gym-macm_amd/csrc include | tar -x -C "$D"
mkdir -p "$D/build"
for f in "$D"/gym-macm_amd/csrc/*.hip; do
  b=$(basename "$f" .hip)
  X=""; [ "$b" = flock_rollout_w64 ] && X="-mllvm -disable-machine-licm"  # as the Makefile
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall \
    -Wno-unused-result $X "$@" -c -o "$D/build/$b.o" "$f" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "ab/$NAME.so" "$D"/build/*.o
rm -rf "$D"
echo "built ab/$NAME.so from $COMMIT"
