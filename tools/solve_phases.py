"""Phase split of the split step's solver kernel (flock_solve_wg) from the diagnostic
stamp build: velocity (warm start + iterations) vs StoreImpulses + integrate + position.
    make -C gym-macm_amd stamps && python tools/solve_phases.py --envs 2048 --agents 1024"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MACM_LIB"] = os.path.join(REPO, "gym-macm_amd", "build", "libmacm_hip_stamps.so")
sys.path.insert(0, os.path.join(REPO, "gym-macm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_macm import _abi  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=2048)
ap.add_argument("--agents", type=int, default=1024)
ap.add_argument("--flocks", type=int, default=1)
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()
L = _abi.lib()
L.macm_debug_stamps.restype = ctypes.c_int
L.macm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
E, N = a.envs, a.agents
targets = None if a.flocks <= 1 else [i * a.flocks // N for i in range(N)]
vec = FlockVec(E, n_agents=[N], targets=targets, seed=0x6D61636D, device="cuda:0")
gen = torch.Generator(device="cuda:0")
gen.manual_seed(1)
buf = np.zeros((E, 16), np.uint64)
vel, rest = [], []
for s in range(a.warmup + a.steps):
    act = torch.randint(0, 3, (E, N, 3), dtype=torch.uint8, device="cuda:0", generator=gen)
    vec.step(act)
    if s >= a.warmup:
        torch.cuda.synchronize()
        _abi.check(L.macm_debug_stamps(vec.world.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))), "stamps")
        t = buf[:, 13:16].astype(np.int64)
        vel.append(t[:, 1] - t[:, 0])
        rest.append(t[:, 2] - t[:, 1])
v, r = np.concatenate(vel), np.concatenate(rest)
print(f"solver cycles per env: velocity mean {v.mean():.0f} max {v.max()}, store+integrate+position mean {r.mean():.0f} max {r.max()}")
