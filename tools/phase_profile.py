"""Per-phase cycle shares of flock_step_w64 from the diagnostic stamp build.

    make -C gym-macm_amd stamps && python tools/phase_profile.py [--envs 4096] [--steps 20]

Loads build/libmacm_hip_stamps.so (in-kernel s_memtime at phase boundaries; see
STAMP() in csrc/flock_step_w64.hip). Read SHARES, not absolute time: the stamps'
s_waitcnt(0) forbids overlaps the product kernel has.
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
from gym_macm.vec import FlockVec  # noqa: E402

PHASES = ["actions", "collide", "adjacency", "dfs+integrate+normals", "velocity_solve", "integrate_pos",
          "position_solve+sleepclk", "sleep_decision", "sync_fixtures", "pairs+nearest", "list_build",
          "reward+obs+writeback", "bookkeeping"]
# flock_step_wg (N > 64): WSTAMP(0..12) in csrc/flock_step_wg.hip
# split step: flock_step_wg_c stamps 0..9, flock_solve_wg stamps 13..15
PHASES_C = ["oldc+sleep_clock", "island_sleep", "sync_fixtures", "grid_build", "pair_sweep+nearest",
            "new_pairs", "old_list", "reward+obs", "writeback"]
PHASES_B = ["solve_velocity", "solve_position"]
PHASES_A = ["A:actions", "A:collide", "A:csr+sort", "A:dfs+levels", "A:level_sort", "A:records"]
PHASES_D = ["A2:dfs+levels", "A2:level_sort+records"]  # flock_dfs_wg (dense envs)
PHASES_WG = ["loads+actions", "collide", "csr+sort", "dfs", "integrate+records", "velocity_solve",
             "impulses+integrate+position", "sleep", "sync_fixtures", "pairs+nearest", "list_build",
             "reward+obs+writeback"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--spread", type=float, default=20.0)
    ap.add_argument("--policy", choices=("random", "bots"), default="random")
    ap.add_argument("--flocks", type=int, default=1, help="targets = i * flocks // N (config 3: 4)")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    L = _abi.lib()
    L.macm_debug_stamps.restype = ctypes.c_int
    L.macm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    E, N = args.envs, args.agents
    targets = None if args.flocks <= 1 else [i * args.flocks // N for i in range(N)]
    vec = FlockVec(E, n_agents=[N], targets=targets, seed=0x6D61636D, device="cuda:0", start_spread=args.spread)
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(1)
    buf = np.zeros((E, 32), np.uint64)
    deltas, stats, walls, stats_wg = [], [], [], []
    for s in range(args.warmup + args.steps):
        if args.policy == "bots":
            from gym_macm.bots import flock_actions
            a = flock_actions(vec.obs)
        else:
            a = torch.randint(0, 3, (E, N, 3), dtype=torch.uint8, device="cuda:0", generator=gen)
        if s >= args.warmup:
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        vec.step(a)
        if s >= args.warmup:
            ev1.record()
            torch.cuda.synchronize()
            walls.append(ev0.elapsed_time(ev1))
            _abi.check(L.macm_debug_stamps(vec.world.h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))),
                       "stamps")
            if N > 64:
                t = np.concatenate([buf[:, :10], buf[:, 13:16]], 1).astype(np.int64)
                dd = np.diff(t, axis=1)
                da = np.diff(buf[:, 16:23].astype(np.int64), axis=1)
                # flock_dfs_wg (dense envs' DFS kernel, stamps 26..28; zero for the envs kernel A walked)
                d2 = np.where(buf[:, 26:27] > 0, np.diff(buf[:, 26:29].astype(np.int64), axis=1), 0)
                deltas.append(np.concatenate([da, dd[:, :9], dd[:, 10:], d2], 1))
            else:
                b16 = buf.reshape(-1)[:E * 16].reshape(E, 16)
                t = b16[:, :14].astype(np.int64)
                deltas.append(np.diff(t, axis=1))
            stats.append(buf.reshape(-1)[:E * 16].reshape(E, 16)[:, 14:].copy())
            stats_wg.append(np.concatenate([buf[:, 10:13], buf[:, 24:26]], 1).copy())
    d = np.concatenate(deltas)  # [steps*E, 13]
    phases = PHASES if N <= 64 else PHASES_A + PHASES_C + PHASES_B + PHASES_D
    st = np.concatenate(stats)
    total = d.sum(axis=1)
    out = {"envs": E, "agents": N, "spread": args.spread, "policy": args.policy, "kernel_ms_stamped": float(np.mean(walls)),
           "wave_cycles_mean": float(total.mean()), "wave_cycles_p95": float(np.percentile(total, 95)),
           "wave_cycles_max": float(total.max()), "phases": {}}
    for k, name in enumerate(phases):
        col = d[:, k]
        out["phases"][name] = {"mean": float(col.mean()), "p95": float(np.percentile(col, 95)),
                               "max": float(col.max()), "share": float(col.sum() / total.sum())}
    if N > 64:  # grid diagnostics of the stamp build (flock_step_wg_c, slots 10..12)
        g = np.concatenate(stats_wg)
        out["grid"] = {"tile_candidates_per_body": float(g[:, 0].mean() / 1000),
                       "bodies_walking_all_strips": float(g[:, 1].mean()),
                       "gs_levels_mean": float((g[:, 2] & 0xFFFFFFFF).mean()),
                       "gs_levels_max": float((g[:, 2] & 0xFFFFFFFF).max()),
                       "touching_mean": float((g[:, 2] >> 32).mean()),
                       "touching_max": float((g[:, 2] >> 32).max())}
        isl = g[:, 4] > 0  # envs that took kernel A's islands-first path: union-find cycles and rounds
        if isl.any():
            out["island_labeling"] = {"envs_frac": float(isl.mean()), "cycles_mean": float(g[isl, 3].mean()),
                                      "cycles_max": float(g[isl, 3].max()), "rounds_mean": float(g[isl, 4].mean()),
                                      "rounds_max": int(g[isl, 4].max())}
        # the launch-boundary tail. Per env and step, the cycles of each kernel (A, the
        # dense envs' DFS kernel, B, C); every launch waits for its slowest env (sum over steps of the
        # per-kernel maxima; with the B -> C handoff, B and C of an env run back to back) against a
        # per-env pipeline that never waits for another env (max over envs of the env's own sum)
        dk = d.reshape(args.steps, E, -1)
        nA, nC, nB = len(PHASES_A), len(PHASES_C), len(PHASES_B)
        kA = dk[:, :, :nA].sum(2)
        kC = dk[:, :, nA:nA + nC].sum(2)
        kB = dk[:, :, nA + nC:nA + nC + nB].sum(2)
        kD = dk[:, :, nA + nC + nB:].sum(2)
        per_launch = float((kA.max(1) + kD.max(1) + kB.max(1) + kC.max(1)).sum())
        handoff = float((kA.max(1) + kD.max(1) + (kB + kC).max(1)).sum())
        piped = float((kA + kD + kB + kC).sum(0).max())
        deepest = int((kA + kD + kB + kC).sum(0).argmax())
        out["pipeline"] = {
            "steps": args.steps,
            "per_launch_cycles": per_launch, "handoff_cycles": handoff, "per_env_pipeline_cycles": piped,
            "pipeline_gain_bound_vs_handoff": 1.0 - piped / handoff,
            "pipeline_gain_bound_vs_per_launch": 1.0 - piped / per_launch,
            "deepest_env": deepest,
            "deepest_env_kernel_cycles": {"A": float(kA[:, deepest].sum()), "DFS": float(kD[:, deepest].sum()),
                                          "B": float(kB[:, deepest].sum()), "C": float(kC[:, deepest].sum())},
            "kernel_max_cycles_sum": {"A": float(kA.max(1).sum()), "DFS": float(kD.max(1).sum()),
                                      "B": float(kB.max(1).sum()), "C": float(kC.max(1).sum())},
        }
        print(json.dumps(out, indent=1))
        if args.json:
            with open(args.json, "w") as f:
                json.dump(out, f, indent=1)
        return
    T = (st[:, 0] & 0xFFFF).astype(np.int64)
    nisl = ((st[:, 0] >> 16) & 0xFFFF).astype(np.int64)
    M = (st[:, 0] >> 32).astype(np.int64)
    maxisl = (st[:, 1] & 0xFFFFFFFF).astype(np.int64)
    cnt = (st[:, 1] >> 32).astype(np.int64)
    for name, v in (("touching", T), ("islands", nisl), ("list_in", M), ("max_island_contacts", maxisl),
                    ("list_out", cnt)):
        out[name] = {"mean": float(v.mean()), "p95": float(np.percentile(v, 95)), "max": int(v.max())}
    # the tail: the slowest 1% of waves (they set the kernel's duration), phase by phase
    slow = total >= np.percentile(total, 99)
    out["slowest_1pct"] = {"waves": int(slow.sum()), "wave_cycles_mean": float(total[slow].mean()),
                           "phases": {name: float(d[slow, k].mean()) for k, name in enumerate(phases)},
                           "touching": float(T[slow].mean()), "islands": float(nisl[slow].mean()),
                           "list_in": float(M[slow].mean()), "max_island_contacts": float(maxisl[slow].mean())}
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
