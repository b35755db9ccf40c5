#!/bin/bash
# Build a variant of libmacm_hip.so from a patched copy of the sources (A/B timing, tools/ab_m.sh):
#   tools/build_src_variant.sh NAME FILE 'old text' 'new text'   ->  abv/NAME.so
set -eu
cd "$(dirname "$0")/.."
NAME=$1 FILE=$2
R=$(mktemp -d)
T=$R/w
mkdir -p "$T" && cp -r gym-macm_amd/csrc gym-macm_amd/Makefile "$T/" && ln -s "$PWD/include" "$R/include"
python3 - "$T/csrc/$FILE" "$3" "$4" <<'PY'
import sys
p, a, b = sys.argv[1:4]
s = open(p).read()
assert s.count(a) == 1, f"{a!r} not found exactly once in {p}"
open(p, "w").write(s.replace(a, b))
PY
(cd "$T" && make -s -j8 >/dev/null)
mkdir -p abv && cp "$T/libmacm_hip.so" "abv/$NAME.so" && rm -rf "$R"
echo "built abv/$NAME.so"
