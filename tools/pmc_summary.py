"""Summarise rocprofv3 PMC passes (tools/pmc.sh) for the step kernel into a JSON
that bench.py reads for `roofline.traffic`.

    python tools/pmc_summary.py gpurun_out/<dir> --envs 4096 --agents 64 -o profiles/pmc_flock_step.json
    python tools/pmc_summary.py gpurun_out/<dir> --kernel "env_step_w64<1, 32, float, false>" --agents 32 \
        -o profiles/pmc_tdm_step.json

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE
and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read, so reads are doubled; WRITE_SIZE is taken as is. The step kernel's
accesses are 1-16 B per lane (uncalibrated widths per the guide), so the figure
is reported together with both raw counters.
"""
import argparse
import collections
import csv
import json
import os


def kernel_means(path, kernel, last=False):
    """Mean per dispatch of each counter over the kernel's dispatches (last: the last dispatch only,
    e.g. the timed rollout launch after the warm-up one)."""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]][r.get("Dispatch_Id", "0")] += float(r["Counter_Value"])
    out = {}
    for k, per in agg.items():
        vals = [per[d] for d in sorted(per, key=lambda x: int(x))]
        out[k] = vals[-1] if last else sum(vals) / len(vals)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="env_step_w64<0, 64, float, true>")
    ap.add_argument("--policy", default="random")
    ap.add_argument("--outputs", default="trajectory", choices=("trajectory", "overwrite"),
                    help="bench.py --outputs of the profiled run (a rollout launch's output form)")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=64)
    ap.add_argument("--steps-per-launch", type=int, default=1,
                    help="env steps one launch of the kernel takes (a rollout launch: its K)")
    ap.add_argument("--last", action="store_true", help="the kernel's last dispatch only")
    ap.add_argument("--commit", default="", help="the commit the profiled library was built from")
    ap.add_argument("-o", "--out", default="")
    a = ap.parse_args()
    # the library the passes ran (lib.sha256, written on the box by tools/pmc.sh): bench.py quotes the
    # traffic only while it loads a library with this hash (no stale PMC in the line)
    lib_sha = None
    sp = os.path.join(a.dir, "lib.sha256")
    if os.path.exists(sp):
        with open(sp) as f:
            lib_sha = f.read().split()[0]
    res = {}
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2"):
        p = os.path.join(a.dir, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            res.update(kernel_means(p, a.kernel, a.last))
    fetch_b = res["FETCH_SIZE"] * 1024.0
    write_b = res["WRITE_SIZE"] * 1024.0
    agents = a.envs * a.agents
    out = {
        "kernel": a.kernel, "envs": a.envs, "agents": a.agents, "policy": a.policy, "outputs": a.outputs,
        "fetch_size_kib": res["FETCH_SIZE"], "write_size_kib": res["WRITE_SIZE"],
        "hbm_bytes_per_launch": 2.0 * fetch_b + write_b,
        "steps_per_launch": a.steps_per_launch,
        "hbm_bytes_per_agent_step": (2.0 * fetch_b + write_b) / agents / a.steps_per_launch,
        "correction": "reads = 2 x FETCH_SIZE (gfx950 half-count), writes = WRITE_SIZE",
        "per_wave": {k: v / res.get("SQ_WAVES", 1.0) for k, v in res.items() if k.startswith("SQ_")},
        "source": a.dir,
        "lib_sha256": lib_sha,
        "commit": a.commit or None,
    }
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
