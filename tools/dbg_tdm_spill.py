"""Debug: first step where a crowded TDM world departs from the oracle (obs / state), and whether
that env took the spill step on that step. Usage: python tools/dbg_tdm_spill.py [--force]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "gym-macm_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_macm import _abi  # noqa: E402
from test_gpu_tdm import make_pair, random_actions  # noqa: E402


def main():
    force = "--force" in sys.argv
    teams, side, seed, steps = [32, 32], 3.0, 5, 60
    E, N = 4, 64
    w, orc = make_pair(E, teams, seed=seed, world_width=side, world_height=side)
    if force:
        w.set_debug(_abi.DEBUG_FORCE_SPILL)
    rng = np.random.default_rng(seed)
    for t in range(steps):
        a = random_actions(rng, E, N, p_attack=0.3)
        s0 = w.spilled()
        w.step(torch.from_numpy(a).cuda())
        r = orc.step(a)
        s1 = w.spilled()
        g = w.get_state()
        o = orc.get_state()
        gobs = w.obs.cpu().numpy()
        ref = r["obs"].astype(np.float32)
        ulp = np.abs(gobs.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
        bad = ulp > 1
        bad_env = [e for e in range(E) if bad[e].any()]
        st_bad = {k: [e for e in range(E) if not np.array_equal(g[k][e], o[k][e])]
                  for k in ("pos", "vel", "angle", "fat", "sleep", "health", "alive", "cd_atk", "cd_mov")}
        st_bad = {k: v for k, v in st_bad.items() if v}
        print(f"step {t}: spilled +{s1 - s0} obs-bad envs {bad_env} state-bad {st_bad}", flush=True)
        if bad_env or st_bad:
            e = (bad_env or list(st_bad.values())[0])[0]
            idx = np.argwhere(bad[e])
            print("  first bad obs entries (agent, slot, comp):", idx[:12].tolist())
            i, j, c = idx[0]
            print("  gpu", gobs[e, i, j], "ref", r["obs"][e, i, j])
            print("  alive", g["alive"][e].sum(), "gpu pos", g["pos"][e, i], "ref pos", o["pos"][e, i])
            print("  gpu angle", g["angle"][e, i], "ref angle", o["angle"][e, i])
            print("  count gpu", g["contact_count"][e], "ref", o["contact_count"][e])
            break


if __name__ == "__main__":
    main()
