#!/bin/bash
# Build a variant of libmacm_hip.so from a patched copy of the sources (A/B timing, tools/ab_m.sh):
#   tools/build_src_variant.sh NAME FILE 'old text' 'new text' ['old text' 'new text' ...]  ->  abv/NAME.so
set -eu
cd "$(dirname "$0")/.."
NAME=$1 FILE=$2
R=$(mktemp -d)
T=$R/w
mkdir -p "$T" && cp -r gym-macm_amd/csrc gym-macm_amd/Makefile "$T/" && ln -s "$PWD/include" "$R/include"
shift 2
python3 - "$T/csrc/$FILE" "$@" <<'PY'
import sys
p, pairs = sys.argv[1], sys.argv[2:]
s = open(p).read()
for a, b in zip(pairs[0::2], pairs[1::2]):
    assert s.count(a) == 1, f"{a!r} not found exactly once in {p}"
    s = s.replace(a, b)
open(p, "w").write(s)
PY
(cd "$T" && make -s -j8 >/dev/null)
mkdir -p abv && cp "$T/libmacm_hip.so" "abv/$NAME.so" && rm -rf "$R"
echo "built abv/$NAME.so"
