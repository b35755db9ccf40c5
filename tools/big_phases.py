"""Phase cycles of the spill step in worlds above 1024 agents (diagnostic stamp build; SSTAMP in
csrc/flock_spill.hpp, stamps 16..27 of each env's row):
    MACM_STAMPS_LIB=abv/stamps.so python tools/big_phases.py --agents 2048 --envs 64 --steps 3"""
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
from gym_macm.vec import FlockVec  # noqa: E402

PH = ["loads+actions", "collide", "csr", "island_dfs (thread 0)", "integrate+records", "velocity (thread/island)",
      "integrate_pos", "position (thread/island)", "sleep+sync", "all-pairs sweep", "list+obs+writeback"]
ap = argparse.ArgumentParser()
ap.add_argument("--agents", type=int, default=2048)
ap.add_argument("--envs", type=int, default=64)
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--json", default="")
a = ap.parse_args()
L = _abi.lib()
L.macm_debug_stamps.restype = ctypes.c_int
L.macm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
E, N = a.envs, a.agents
vec = FlockVec(E, n_agents=[N], seed=0x6D61636D, device="cuda:0")
g = torch.Generator(device="cuda:0")
g.manual_seed(1)
buf = np.zeros((E, 32), np.uint64)
rows = []
for s in range(a.warmup + a.steps):
    vec.step(torch.randint(0, 3, (E, N, 3), dtype=torch.uint8, device="cuda:0", generator=g))
    if s >= a.warmup:
        torch.cuda.synchronize()
        _abi.check(L.macm_debug_stamps(vec.world.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))), "stamps")
        rows.append(np.diff(buf[:, 16:28].astype(np.int64), axis=1))
d = np.concatenate(rows)
tot = d.sum(1)
out = {"agents": N, "envs": E, "cycles_mean": float(tot.mean()), "cycles_max": float(tot.max()),
       "phases": {p: {"mean": float(d[:, k].mean()), "max": float(d[:, k].max()), "share": float(d[:, k].sum() / tot.sum())}
                  for k, p in enumerate(PH)}}
print(json.dumps(out, indent=1))
if a.json:
    with open(a.json, "w") as f:
        json.dump(out, f, indent=1)
