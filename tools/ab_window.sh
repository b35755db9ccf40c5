#!/bin/bash
# Driver-window repeats (--steps 20 --warmup 5) of library variants: tools/ab_window.sh OUT lib... -- bench args
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ $# -gt 0 ] && shift
for r in 1 2 3; do
  for i in "${!LIBS[@]}"; do
    MACM_LIB="$PWD/${LIBS[$i]}" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/v${i}_r$r.json" 2>/dev/null || exit $?
  done
done
python3 - "$OUT" "${LIBS[@]}" <<'PY'
import json, sys, glob
out, libs = sys.argv[1], sys.argv[2:]
for i, l in enumerate(libs):
    v = []
    for f in sorted(glob.glob(f"{out}/v{i}_r*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        v.append((round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["kernel_ms"] * 1e3, 1)))
    print(l, "(us/step, kernel us):", v)
PY
echo ALLDONE
