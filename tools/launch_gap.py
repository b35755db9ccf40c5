"""How much of a step is launch overhead? The metric config's driver window (steps 6..25 from
reset) stepped three ways on one world, each from the same reset and actions:

  loop   one macm_world_step per step from Python (what bench.py times)
  graph  the 20 steps captured once into a HIP graph (torch.cuda.CUDAGraph), replayed
  empty  a trivial 4096-workgroup kernel launched back to back (the floor of a launch)

and checks that loop and graph leave bit-identical state.

    python tools/launch_gap.py [--envs 4096] [--agents 64] [--warmup 5] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gym-macm_amd"))

import torch  # noqa: E402

from gym_macm.vec import FlockVec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--flocks", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    E, N, W, K = args.envs, args.agents, args.warmup, args.steps
    seed = 0x6D61636D
    targets = None if args.flocks <= 1 else [i * args.flocks // N for i in range(N)]
    vec = FlockVec(E, n_agents=[N], targets=targets, seed=seed, device=dev)
    w = vec.world
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed + 1)
    acts = torch.randint(0, 3, (W + K, E, N, 3), dtype=torch.uint8, device=dev, generator=gen)
    stride = E * N * 3
    base = acts.data_ptr()
    res = {"envs": E, "agents": N, "flocks": args.flocks, "warmup": W, "steps": K}

    def warm(stream):
        w.reset(seed, 0)
        for k in range(W):
            w.step_raw(base + k * stride, stream.cuda_stream)
        torch.cuda.synchronize()

    # loop: as bench.py
    s0 = torch.cuda.current_stream(dev)
    loop_us = []
    for _ in range(args.reps):
        warm(s0)
        t0 = time.perf_counter()
        for k in range(K):
            w.step_raw(base + (W + k) * stride, s0.cuda_stream)
        torch.cuda.synchronize()
        loop_us.append((time.perf_counter() - t0) / K * 1e6)
    ref = [t.clone() for t in (w.obs, w.nbr_id, w.reward)]
    res["loop_us_per_step"] = loop_us

    # graph: capture K steps (an even count keeps the world's double-buffer parity), replay
    assert K % 2 == 0
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(dev)
    warm(s0)
    with torch.cuda.graph(g, stream=cs):
        st = torch.cuda.current_stream(dev).cuda_stream
        for k in range(K):
            w.step_raw(base + (W + k) * stride, st)
    graph_us = []
    for r in range(args.reps):
        warm(s0)
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        graph_us.append((time.perf_counter() - t0) / K * 1e6)
        if r == 0:
            same = all(torch.equal(a, b) for a, b in zip(ref, (w.obs, w.nbr_id, w.reward)))
            res["graph_matches_loop"] = bool(same)
    res["graph_us_per_step"] = graph_us

    # streams: the same E envs as S worlds of E/S envs (env_offset: env e is the same env), each
    # stepped on its own stream, so one slice's next step overlaps another's tail
    for S in (2, 4):
        if E % S:
            continue
        Es = E // S
        subs = [FlockVec(Es, n_agents=[N], targets=targets, seed=seed, env_offset=i * Es, device=dev).world
                for i in range(S)]
        strs = [torch.cuda.Stream(dev) for _ in range(S)]
        sacts = [acts[:, i * Es:(i + 1) * Es].contiguous() for i in range(S)]
        sstride = Es * N * 3
        su = []
        for _ in range(args.reps):
            for i in range(S):
                subs[i].reset(seed, i * Es)
                for k in range(W):
                    subs[i].step_raw(sacts[i].data_ptr() + k * sstride, strs[i].cuda_stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                for i in range(S):
                    subs[i].step_raw(sacts[i].data_ptr() + (W + k) * sstride, strs[i].cuda_stream)
            torch.cuda.synchronize()
            su.append((time.perf_counter() - t0) / K * 1e6)
        res[f"streams{S}_us_per_step"] = su
        res[f"streams{S}_matches_loop"] = bool(all(
            torch.equal(torch.cat([getattr(sw, nm) for sw in subs]), r)
            for nm, r in zip(("obs", "nbr_id", "reward"), ref)))
        del subs

    # empty: the cost of a 4096-workgroup launch that does (almost) nothing
    x = torch.zeros(E * 64, device=dev)
    for _ in range(50):
        x.add_(1.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(1000):
        x.add_(1.0)
    torch.cuda.synchronize()
    res["empty_us_per_launch"] = (time.perf_counter() - t0) / 1000 * 1e6
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
