"""Summarise tools/ab_multi.sh output: per config and variant, the median ms_per_step of the 3 runs."""
import glob, json, os, re, statistics, sys
d = sys.argv[1]
rows = {}
for p in glob.glob(os.path.join(d, "*_v*_r*.json")):
    m = re.match(r"(.+)_v(\d+)_r(\d+)\.json", os.path.basename(p))
    try:
        j = json.load(open(p))
    except Exception:
        continue
    rows.setdefault(m.group(1), {}).setdefault(int(m.group(2)), []).append(j["ms_per_step"] * 1e3)
for cfg, v in sorted(rows.items()):
    meds = {k: statistics.median(x) for k, x in v.items()}
    base = meds.get(0)
    print(cfg.ljust(12), "  ".join(f"v{k}: {meds[k]:9.2f} us ({(meds[k] / base - 1) * 100:+.1f}%) {sorted(round(x, 1) for x in v[k])}"
                                    for k in sorted(meds)))
