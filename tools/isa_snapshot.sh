#!/bin/bash
# Device assembly of every translation unit of libmacm_hip.so with the product flags, into $1
# (default tools/build/isa): diff two snapshots to prove a source change leaves the gfx950 code
# unchanged (e.g. deleting A/B knobs and the variants they selected).
set -eu
OUT=$(realpath -m "${1:-$(dirname "$0")/build/isa}")
mkdir -p "$OUT"
cd "$(dirname "$0")/../gym-macm_amd"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-result"
for f in csrc/*.hip; do
  b=$(basename "$f" .hip)
  extra=""
  [ "$b" = flock_rollout_w64 ] && extra="-mllvm -disable-machine-licm"
  /opt/rocm/bin/hipcc $FLAGS $extra --cuda-device-only -S -o "$OUT/$b.s" "$f" &
done
wait
# the assembly without comments, file names and the per-TU module id, for diffing
for s in "$OUT"/*.s; do
  grep -v '^\s*;' "$s" | grep -v '\.file\|\.ident\|__hip_cuid_\|amdhsa.target\|^\s*$' > "${s%.s}.isa"
done
echo "$OUT"
