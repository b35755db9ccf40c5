"""Print tools/phase_wg.sh results side by side: python tools/phase_show.py DIR variant ..."""
import json
import sys

d, vs = sys.argv[1], sys.argv[2:]
for c in ("c3", "c5", "c3b"):
    res = {}
    for v in vs:
        try:
            res[v] = json.load(open(f"{d}/{c}_{v}.json"))
        except Exception:  # noqa: BLE001
            pass
    if not res:
        continue
    print(f"{c}: " + "  ".join(f"{v} {r['kernel_ms_stamped']:.3f} ms" for v, r in res.items()))
    names = list(next(iter(res.values()))["phases"])
    for n in names:
        print(f"   {n:22s}" + "".join(f" {r['phases'][n]['mean']:11.0f}" for r in res.values()))
    for v, r in res.items():
        if "grid" in r:
            print(f"   grid[{v}]: " + ", ".join(f"{k} {x:.3g}" for k, x in r["grid"].items()))
