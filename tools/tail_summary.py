"""Medians of tools/tail_ab.sh runs: python tools/tail_summary.py gpurun_out/<dir>"""
import collections
import glob
import json
import re
import statistics
import sys

d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*.json"):
    n = f.split("/")[-1][:-5]
    m = re.match(r"(.*)_(v\w+)_r\d", n)
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        print("unreadable", f)
        continue
    d[(m.group(1), m.group(2))].append(j["ms_per_step"] * 1e3)
for k in sorted(d):
    print("%-18s %-8s median %7.2f us  %s" % (k[0], k[1], statistics.median(d[k]), [round(x, 2) for x in sorted(d[k])]))
