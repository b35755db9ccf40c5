#!/bin/bash
# TDM obs writer A/B: time (C4, 3 alternations) and WRITE_SIZE per launch for each library.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for r in 1 2 3; do
  i=0
  for lib in "$@"; do
    MACM_LIB="$R/$lib" timeout -k 10 120 python bench.py --env tdm --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/v${i}_r$r.json" 2>/dev/null || exit $?
    i=$((i + 1))
  done
done
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  export MACM_LIB="$R/$lib"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$R/$OUT/pmc_v$i" -o run -- \
    python3 "$R/bench.py" --env tdm --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2>&1 || exit $?
  i=$((i + 1))
done
cd "$R"
python3 - "$OUT" "$@" <<'PY'
import sys, glob, json, csv, collections
out, libs = sys.argv[1], sys.argv[2:]
for i, lib in enumerate(libs):
    ts = []
    for f in glob.glob(f"{out}/v{i}_r*.json"):
        ts.append(json.loads(open(f).read().strip().splitlines()[0])["ms_per_step"] * 1e3)
    w = []
    for f in glob.glob(f"{out}/pmc_v{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "env_step_w64" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
                w.append(float(r["Counter_Value"]))
    wmb = sum(w) / len(w) * 1024 / 1e6 if w else float("nan")
    print(f"v{i} {lib}: {min(ts):.2f} us/step (min of {len(ts)}), WRITE_SIZE {wmb:.1f} MB per launch "
          f"= {wmb * 1e6 / (4096 * 32):.0f} B per agent-step")
PY
echo ALLDONE
