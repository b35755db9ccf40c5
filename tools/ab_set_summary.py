"""Summarise tools/ab_set.sh: per workload and variant, us per step of the timed window (host clock,
the bench line's ms_per_step) and the per-step kernel time on the launch stream; min over reps."""
import glob
import json
import os
import re
import sys

for d in sys.argv[1:]:
    res = {}
    for f in sorted(glob.glob(os.path.join(d, "*_v*_r*.json"))):
        m = re.match(r"(.+)_v(\d+)_r(\d+)\.json", os.path.basename(f))
        try:
            j = json.loads(open(f).read().strip().split("\n")[-1])
        except Exception as e:  # noqa: BLE001
            print(f, "unreadable:", e)
            continue
        res.setdefault((m.group(1), int(m.group(2))), []).append((j["ms_per_step"] * 1e3, j["value"] / 1e9))
    for (w, v), x in sorted(res.items()):
        us = [a for a, _ in x]
        print(f"{w:7s} v{v}  " + " ".join(f"{a:9.2f}" for a in us) + f"   min {min(us):9.2f} us/step "
              f"({max(b for _, b in x):.3f} G agent-steps/s)")
