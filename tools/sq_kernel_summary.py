"""Per-kernel SQ counter summary of rocprofv3 --pmc passes (tools/gpu_final_r05.sh sq_* dirs): for each
kernel, the counters summed over its dispatches, per wave (÷ SQ_WAVES of the same pass set), and the
ratios the round's analysis uses (wait cycles per VALU-active cycle, VALU instructions per wave).
    python tools/sq_kernel_summary.py profiles/r05/final/sq_c5_1 profiles/r05/final/sq_c5_2"""
import collections
import csv
import os
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k.startswith("__amd") or "at::" in k:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((d, r.get("Dispatch_Id", "0")))
for k in sorted(tot):
    c = tot[k]
    waves = c.get("SQ_WAVES", 0.0)
    line = [f"{k}: dispatches {len(disp[k])}"]
    if waves:
        line.append(f"waves {waves:.0f}")
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_LDS"):
            if n in c:
                line.append(f"{n}/wave {c[n] / waves:.0f}")
    if c.get("SQ_ACTIVE_INST_VALU"):
        line.append(f"SQ_WAIT_ANY/SQ_ACTIVE_INST_VALU {c.get('SQ_WAIT_ANY', 0) / c['SQ_ACTIVE_INST_VALU']:.2f}")
    print("; ".join(line))
