"""Summarise tools/ab.sh results: kernel µs per variant per repetition (min is the robust figure)."""
import glob
import json
import os
import sys

for d in sys.argv[1:]:
    res = {}
    for f in sorted(glob.glob(os.path.join(d, "v*_r*.json"))):
        v = os.path.basename(f).split("_")[0]
        try:
            j = json.loads(open(f).read().strip().split("\n")[-1])
        except Exception as e:  # noqa: BLE001
            print(f, "unreadable:", e)
            continue
        res.setdefault(v, []).append(j["roofline"]["kernel_ms"] * 1000)
    for v, x in sorted(res.items()):
        print(f"{d} {v} " + " ".join(f"{t:8.2f}" for t in x) + f"   min {min(x):8.2f} us")
