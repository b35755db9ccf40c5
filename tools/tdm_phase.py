"""Per-phase cycles of the TDM wave kernel (env_step_w64<kTdm>) from the diagnostic stamp build.

    make -C gym-macm_amd stamps && python tools/tdm_phase.py [--envs 512] [--teams 16,16]

One launch per step (macm_tdm_step); lane 0 of each env's wave records s_memtime at the phase
boundaries (STAMP() in csrc/flock_step_w64.hip). The stamps' s_waitcnt(0) forbid overlaps the
product kernel has: read SHARES and per-wave cycles, not absolute time.
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MACM_LIB"] = os.environ.get("MACM_STAMPS_LIB",
                                        os.path.join(REPO, "gym-macm_amd", "build", "libmacm_hip_stamps.so"))
sys.path.insert(0, os.path.join(REPO, "gym-macm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_macm import _abi  # noqa: E402
from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402

PHASES = ["loads+actions+raycasts", "collide", "adjacency", "dfs+integrate+normals", "velocity_solve",
          "integrate_pos", "position_solve+sleepclk", "sleep_decision", "sync_fixtures", "pairs+nearest",
          "list_build", "writeback+obs", "bookkeeping"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=512)
    ap.add_argument("--teams", default="16,16")
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    L = _abi.lib()
    L.macm_debug_tdm_stamps.restype = ctypes.c_int
    L.macm_debug_tdm_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    E = args.envs
    teams = [int(x) for x in args.teams.split(",")]
    N = sum(teams)
    w = TdmWorld(tdm_config(teams), E, device="cuda:0")
    w.reset(0x6D61636D, 0)
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(1)
    buf = np.zeros((E, 32), np.uint64)
    deltas, walls = [], []
    for s in range(args.warmup + args.steps):
        a = torch.randint(0, 3, (E, N, 4), dtype=torch.uint8, device="cuda:0", generator=gen)
        a[..., 3] = torch.randint(0, 2, (E, N), dtype=torch.uint8, device="cuda:0", generator=gen)
        if s >= args.warmup:
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        w.step(a)
        if s >= args.warmup:
            ev1.record()
            torch.cuda.synchronize()
            walls.append(ev0.elapsed_time(ev1))
            _abi.check(L.macm_debug_tdm_stamps(w.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))), "stamps")
            b16 = buf.reshape(-1)[:E * 16].reshape(E, 16)
            deltas.append(np.diff(b16[:, :14].astype(np.int64), axis=1))
    d = np.concatenate(deltas)
    total = d.sum(axis=1)
    out = {"envs": E, "teams": teams, "kernel_ms_stamped": float(np.mean(walls)),
           "wave_cycles_mean": float(total.mean()), "wave_cycles_p95": float(np.percentile(total, 95)),
           "wave_cycles_max": float(total.max()), "phases": {}}
    for k, name in enumerate(PHASES):
        col = d[:, k]
        out["phases"][name] = {"mean": float(col.mean()), "p95": float(np.percentile(col, 95)),
                               "max": float(col.max()), "share": float(col.sum() / total.sum())}
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
