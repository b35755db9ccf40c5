"""Per-wave SQ counters per macm kernel for tools/pmc_ab.sh variants."""
import collections
import csv
import glob
import sys

out, libs = sys.argv[1], sys.argv[2:]
for i, lib in enumerate(libs):
    print(f"v{i} {lib}")
    path = glob.glob(f"{out}/v{i}/**/*counter_collection.csv", recursive=True)
    if not path:
        print("   no counter file")
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path[0])):
        if "macm" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("macm::", "")
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, c in agg.items():
        m = {k: sum(v) / len(v) for k, v in c.items()}
        w = m.get("SQ_WAVES", 1.0) or 1.0
        print(f"   {name:32s} waves {w:9.0f}  per wave: " +
              "  ".join(f"{k.replace('SQ_', '')} {m[k] / w:9.0f}" for k in sorted(m) if k != "SQ_WAVES"))
