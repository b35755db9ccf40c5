"""One-step field-by-field diff of the workgroup path against the oracle (debug aid).
    python tools/debug_wg.py --agents 100 --envs 6 --seed 100 --spread 12 [--steps 1]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("gym-macm_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from parity import oracle_for  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402
from parity import STATE_KEYS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--agents", type=int, default=100)
ap.add_argument("--envs", type=int, default=6)
ap.add_argument("--seed", type=int, default=100)
ap.add_argument("--spread", type=float, default=12.0)
ap.add_argument("--steps", type=int, default=1)
a = ap.parse_args()
E, N = a.envs, a.agents
kw = dict(start_spread=a.spread)
vec = FlockVec(E, n_agents=[N], seed=a.seed, device="cuda:0", **kw)
cfg = to_config(flockSettings(**kw), N, vec.n_targets, obs_f64=True)
orc = oracle_for(cfg, vec.targets_idx, E, a.seed, 0)
rng = np.random.default_rng(a.seed)
C = vec.world.C
for t in range(a.steps):
    act = rng.integers(0, 3, size=(E, N, 3)).astype(np.uint8)
    vec.step(torch.from_numpy(act).cuda())
    orc.step(act)
    gs, os_ = vec.get_state(), orc.get_state(C)
    print(f"step {t}")
    for k in list(STATE_KEYS) + ["contact_count"]:
        g, o = np.asarray(gs[k]), np.asarray(os_[k])
        bad = np.argwhere(g != o)
        if len(bad):
            print(f"  {k}: {len(bad)} mismatches, first {bad[:4].tolist()}")
            i = tuple(bad[0])
            print(f"     gpu {g[i]!r} oracle {o[i]!r}")
    for e in range(E):
        n = int(gs["contact_count"][e])
        no = int(os_["contact_count"][e])
        if n != no or not np.array_equal(gs["contact_ab"][e, :n], os_["contact_ab"][e, :n]):
            print(f"  env {e}: contact list differs ({n} vs {no})")
        elif not np.array_equal(gs["contact_imp"][e, :n], os_["contact_imp"][e, :n]):
            d = np.argwhere(gs["contact_imp"][e, :n] != os_["contact_imp"][e, :n])
            print(f"  env {e}: impulses differ at {len(d)} entries, first {d[:3].tolist()}")
print("status", vec.status())
