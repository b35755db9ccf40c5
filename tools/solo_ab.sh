#!/bin/bash
# A/B of the solo split (MACM_SOLO_ENVS) on a closed-loop and an open-loop rollout workload, each value in
# a fresh process, alternating, two rounds.  tools/solo_ab.sh OUTNAME "0 32 64" [bench args...]
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/$1; VALS=$2; shift 2
mkdir -p "$OUT"
for round in 1 2; do
  for h in $VALS; do
    MACM_SOLO_ENVS=$h timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/solo${h}_r${round}.json" 2> "$OUT/solo${h}_r${round}.err" || exit $?
    python - "$OUT/solo${h}_r${round}.json" "$h" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"solo {sys.argv[2]:>4}: {j['ms_per_step'] * 1e3:8.1f} us/step host, {j['roofline']['kernel_ms'] * 1e3:8.1f} kernel")
PY
  done
done
