"""Wave timeline of env_step_w64 from the diagnostic MACM_TIMELINE build: when each env's
wave starts and ends (s_memrealtime, 100 MHz, comparable across CUs), its lifetime in
shader cycles (s_memtime) and where it ran (HW_ID / XCC_ID). Answers: how long the
dispatch ramp is, how the waves spread over XCDs / CUs / SIMDs, and how long the tail is.

    tools/build_variant.sh timeline -DMACM_STAMPS -DMACM_TIMELINE
    MACM_LIB=ab/timeline.so python tools/timeline.py [--policy bots] [--json out.json]
"""
import argparse
import collections
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MACM_LIB", os.path.join(REPO, "ab", "timeline.so"))
sys.path.insert(0, os.path.join(REPO, "gym-macm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_macm import _abi  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--policy", choices=("random", "bots"), default="random")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    L = _abi.lib()
    L.macm_debug_stamps.restype = ctypes.c_int
    L.macm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    E, N = args.envs, args.agents
    vec = FlockVec(E, n_agents=[N], seed=0x6D61636D, device="cuda:0")
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(1)
    buf = np.zeros((E, 32), np.uint64)  # macm_debug_stamps copies 32 words per env
    steps = []
    for s in range(args.warmup + args.steps):
        if args.policy == "bots":
            from gym_macm.bots import flock_actions
            a = flock_actions(vec.obs)
        else:
            a = torch.randint(0, 3, (E, N, 3), dtype=torch.uint8, device="cuda:0", generator=gen)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        vec.step(a)
        ev1.record()
        torch.cuda.synchronize()
        if s < args.warmup:
            continue
        _abi.check(L.macm_debug_stamps(vec.world.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))), "stamps")
        b = buf.reshape(-1)[:E * 16].reshape(E, 16).astype(np.int64)  # the wave kernel's stride is 16
        rt0, c0, hw, rt1, c1 = b[:, 0], b[:, 1], b[:, 2], b[:, 3], b[:, 4]
        t0 = rt0 - rt0.min()
        life = c1 - c0
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 7
        xcc = (hw >> 32) & 15
        cu_key = xcc * 1000 + se * 100 + sh * 20 + cu
        simd_key = cu_key * 4 + simd
        per_cu = collections.Counter(cu_key.tolist())
        per_simd = collections.Counter(simd_key.tolist())
        life_simd = collections.defaultdict(int)
        for k, l in zip(simd_key.tolist(), life.tolist()):
            life_simd[k] += l
        steps.append({
            "event_us": ev0.elapsed_time(ev1) * 1e3,
            "span_us": float((rt1.max() - rt0.min()) / 100.0),
            "start_us": {"p50": float(np.percentile(t0, 50) / 100), "p99": float(np.percentile(t0, 99) / 100),
                         "max": float(t0.max() / 100)},
            "end_us": {"p50": float(np.percentile(rt1 - rt0.min(), 50) / 100),
                       "p99": float(np.percentile(rt1 - rt0.min(), 99) / 100),
                       "max": float((rt1 - rt0.min()).max() / 100)},
            "life_cycles": {"mean": float(life.mean()), "p50": float(np.percentile(life, 50)),
                            "p99": float(np.percentile(life, 99)), "max": int(life.max())},
            "clock_ghz": float(np.median(life / np.maximum(rt1 - rt0, 1)) / 10.0),
            "xcds": int(len(set(xcc.tolist()))), "cus": len(per_cu), "simds": len(per_simd),
            "waves_per_cu": {str(k): v for k, v in sorted(collections.Counter(per_cu.values()).items())},
            "waves_per_simd": {str(k): v for k, v in sorted(collections.Counter(per_simd.values()).items())},
            "simd_life_sum_cycles": {"mean": float(np.mean(list(life_simd.values()))),
                                     "max": int(max(life_simd.values()))},
        })
    out = {"envs": E, "agents": N, "policy": args.policy, "steps": steps}
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
