"""Where the host time around bench.py's timed rollout launch goes: the metric
config's driver window (W = 5 warm-up steps, then one 20-step rollout launch) repeated, with the
host-side cost of each call in the timed region measured separately:

  record0  ev0.record(stream) before the launch
  launch   world.rollout_raw (ctypes -> macm_world_rollout -> hipLaunchKernel)
  record1  ev1.record(stream) after it
  sync     torch.cuda.synchronize() until the kernel is done and the host has seen it
  total    the timed region as bench.py measures it; kernel = the event time

    python tools/host_gap.py [--reps 10] [--spin]
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gym-macm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--spin", action="store_true", help="hipSetDeviceFlags(hipDeviceScheduleSpin) first")
    ap.add_argument("--prerecord", action="store_true",
                    help="record both events once and synchronize before the timed launch")
    ap.add_argument("--bench-like", action="store_true",
                    help="between the warm-up and the timed launch, the calls bench.py makes (counter reset, "
                         "spill-count read, a second synchronize)")
    a = ap.parse_args()
    if a.spin:
        ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL).hipSetDeviceFlags(1)
    from gym_macm.vec import FlockVec
    dev = torch.device("cuda:0")
    E, N, W, K, seed = 4096, 64, 5, 20, 0x6D61636D
    vec = FlockVec(E, n_agents=[N], seed=seed, device=dev)
    w = vec.world
    acts = torch.randint(0, 3, (W + K, E, N, 3), dtype=torch.uint8, device=dev,
                         generator=torch.Generator(device=dev).manual_seed(seed + 1))
    stream = torch.cuda.current_stream(dev)
    sh, base, stride = stream.cuda_stream, acts.data_ptr(), E * N * 3
    rows = []
    for r in range(a.reps + 1):
        vec.reset()
        w.rollout_raw(base, W, sh)
        torch.cuda.synchronize(dev)
        if a.bench_like:
            w.reset_counters()
            w.spilled()
            torch.cuda.synchronize(dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if a.prerecord:  # the events' lazy creation outside the timed region
            ev0.record(stream)
            ev1.record(stream)
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record(stream)
        t1 = time.perf_counter()
        w.rollout_raw(base + W * stride, K, sh)
        t2 = time.perf_counter()
        ev1.record(stream)
        t3 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t4 = time.perf_counter()
        row = dict(record0=t1 - t0, launch=t2 - t1, record1=t3 - t2, sync=t4 - t3, total=t4 - t0,
                   kernel=ev0.elapsed_time(ev1) * 1e-3)
        if r:  # the first repetition warms the code paths (bench.py times one window: reported apart)
            rows.append(row)
        else:
            first = {k: round(v * 1e6, 2) for k, v in row.items()}
            first["gap"] = round(first["total"] - first["kernel"], 2)
    med = {k: float(np.median([x[k] for x in rows])) * 1e6 for k in rows[0]}
    med["gap"] = med["total"] - med["kernel"]
    print(json.dumps({"us_median": {k: round(v, 2) for k, v in med.items()}, "us_first": first, "spin": a.spin,
                      "bench_like": a.bench_like, "prerecord": a.prerecord, "reps": a.reps}))


if __name__ == "__main__":
    main()
