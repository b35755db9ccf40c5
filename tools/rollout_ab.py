"""Per-step launches vs one rollout launch (macm_world_rollout / macm_tdm_rollout) over the same
window from the same reset and actions: time per step of each, and whether the rollout leaves
the same state and outputs (bit-exact). MACM_LIB selects the library (tools/build_variant.sh).

    MACM_LIB=ab/roll1.so python tools/rollout_ab.py [--env tdm] [--warmup 5] [--steps 20]
"""
import argparse
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
    ap.add_argument("--env", choices=("flock", "tdm"), default="flock")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--flocks", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    E, W, K = args.envs, args.warmup, args.steps
    seed = 0x6D61636D
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed + 1)
    if args.env == "flock":
        from gym_macm.vec import FlockVec
        N = args.agents
        targets = None if args.flocks <= 1 else [i * args.flocks // N for i in range(N)]
        w = FlockVec(E, n_agents=[N], targets=targets, seed=seed, device=dev).world
        acts = torch.randint(0, 3, (W + K, E, N, 3), dtype=torch.uint8, device=dev, generator=gen)
        outs = lambda: (w.obs, w.nbr_id, w.reward, w.collided, w.done)  # noqa: E731
    else:
        from gym_macm.tdm_world import TdmWorld, tdm_config
        N = 32
        w = TdmWorld(tdm_config([16, 16]), E, device=dev)
        acts = torch.randint(0, 3, (W + K, E, N, 4), dtype=torch.uint8, device=dev, generator=gen)
        acts[..., 3] = torch.randint(0, 2, (W + K, E, N), dtype=torch.uint8, device=dev, generator=gen)
        outs = lambda: tuple(w.outputs())  # noqa: E731
    stride = acts[0].numel()
    base = acts.data_ptr()
    sh = torch.cuda.current_stream(dev).cuda_stream

    def warm():
        w.reset(seed, 0)
        for k in range(W):
            w.step_raw(base + k * stride, sh)
        torch.cuda.synchronize()

    res = {"env": args.env, "envs": E, "agents": N, "warmup": W, "steps": K, "lib": os.environ.get("MACM_LIB", "")}
    loop, roll = [], []
    for _ in range(args.reps):
        warm()
        t0 = time.perf_counter()
        for k in range(K):
            w.step_raw(base + (W + k) * stride, sh)
        torch.cuda.synchronize()
        loop.append((time.perf_counter() - t0) / K * 1e6)
    ref_out = [t.clone() for t in outs()]
    ref_state = w.get_state()
    for _ in range(args.reps):
        warm()
        t0 = time.perf_counter()
        w.rollout_raw(base + W * stride, K, sh)
        torch.cuda.synchronize()
        roll.append((time.perf_counter() - t0) / K * 1e6)
    st = w.get_state()
    res["loop_us_per_step"] = loop
    res["rollout_us_per_step"] = roll
    res["outputs_equal"] = bool(all(torch.equal(a, b) for a, b in zip(ref_out, outs())))
    res["state_equal"] = bool(all(np.array_equal(ref_state[k], st[k]) for k in ref_state))
    res["status"] = int(w.status())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
