"""Summarise tools/kprof.sh output: average microseconds per macm kernel for each variant."""
import csv
import json
import sys

out, libs = sys.argv[1], sys.argv[2:]
for i, lib in enumerate(libs):
    rows = list(csv.DictReader(open(f"{out}/v{i}/run_kernel_stats.csv")))
    try:
        b = json.loads(open(f"{out}/v{i}.json").read().strip().splitlines()[0])
        head = f"{b['ms_per_step'] * 1e3:.1f} us/step (events)"
    except Exception as ex:  # noqa: BLE001
        head = f"no bench line ({ex})"
    print(f"v{i} {lib}: {head}")
    for r in rows:
        if "macm" in r["Name"]:
            name = r["Name"].split("(")[0].replace("void ", "").replace("macm::", "")
            print(f"   {name:40s} calls {r['Calls']:>5s}  avg {float(r['AverageNs']) / 1e3:9.2f} us")
