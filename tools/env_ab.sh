#!/bin/bash
# A/B of an environment knob of the library (e.g. MACM_HANDOFF, MACM_SOLO_ENVS): each value in a fresh
# process, alternating, two rounds.   tools/env_ab.sh OUTNAME VAR "v1 v2 ..." [bench args...]
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/$1; VAR=$2; VALS=$3; shift 3
mkdir -p "$OUT"
for round in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/${VAR}_${v}_r${round}.json" 2> "$OUT/${VAR}_${v}_r${round}.err" || exit $?
    python - "$OUT/${VAR}_${v}_r${round}.json" "$VAR=$v" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>18}: {j['ms_per_step'] * 1e3:9.1f} us/step host, {j['roofline']['kernel_ms'] * 1e3:9.1f} kernel, "
      f"{j['value'] / 1e6:9.1f} M agent-steps/s")
PY
  done
done
