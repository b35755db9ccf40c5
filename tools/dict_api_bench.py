"""Steps/s of the drop-in dict API (gym_macm.envs.Flock / TDM, one env) on cuda:0:
the per-step cost a reference user sees."""
import json
import os
import random
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gym-macm_amd"))


def main():
    import torch  # noqa: F401
    from gym_macm.envs import TDM, Flock

    out = {}
    rng = np.random.default_rng(0)
    for N in (4, 64):
        random.seed(0)
        env = Flock(n_agents=[N], device="cuda:0")
        acts = [{i: rng.integers(0, 3, size=3) for i in range(N)} for _ in range(50)]
        for k in range(20):
            env.step(acts[k % 50])
        t0 = time.perf_counter()
        K = 300
        for k in range(K):
            obs, rew = env.step(acts[k % 50])
        dt = (time.perf_counter() - t0) / K
        out[f"flock_n{N}"] = {"ms_per_step": dt * 1e3, "agent_steps_per_s": N / dt}
    random.seed(0)
    env = TDM(render=False, n_agents=[16, 16], device="cuda:0")
    ids = [a.id for a in env.agents]
    t0 = time.perf_counter()
    K = 300
    for k in range(K):
        a = {i: rng.integers(0, 3, size=4) % np.array([3, 3, 3, 2]) for i in ids if i in env.obs}
        env.step(a)
    dt = (time.perf_counter() - t0) / K
    out["tdm_2x16"] = {"ms_per_step": dt * 1e3, "agent_steps_per_s": 32 / dt}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
