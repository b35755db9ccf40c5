"""Summarise a tools/ab.sh output directory: per variant, the ms_per_step of each round (us) and the median.
   python tools/ab_table.py gpurun_out/<dir> [names...]"""
import glob, json, os, statistics, sys

d = sys.argv[1]
names = sys.argv[2:]
rows = {}
for f in sorted(glob.glob(os.path.join(d, "v*_r*.json"))):
    v = int(os.path.basename(f)[1:].split("_")[0])
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    rows.setdefault(v, []).append(j["ms_per_step"] * 1e3)
base = None
for v in sorted(rows):
    med = statistics.median(rows[v])
    base = med if base is None else base
    nm = names[v] if v < len(names) else f"v{v}"
    print(f"{nm:>10}: " + " ".join(f"{x:9.2f}" for x in rows[v]) + f"  median {med:9.2f} us  ({100 * (med / base - 1):+.1f}%)")
