"""Gauss-Seidel chain floor and launch-boundary tail of a workgroup-path window (a measurement
script). Runs the CPU oracle (oracle/) from reset over a bench window and, per env
and step, takes the level structure of the step's touching contacts (Box2D's
island order, level = 1 + the last earlier level sharing a body; oracle/gs_levels.c): L[e, k]
levels per pass.

Kernel B (flock_solve_wg, one wave per env) steps every level of every pass: warm start + vel_iters
velocity passes and up to pos_iters position passes, so env e's chain in step k is
    L[e, k] * ((1 + vel_iters) * c_vel + pos_passes * c_pos)        cycles
with c_vel / c_pos the cycles of one velocity / position level step. With c = the dependent-VALU
floors of the microbenchmark (tools/ubench_level.hip V3 / V14, one wave alone on its SIMD) that is
the chain FLOOR of bit-exact Gauss-Seidel in Box2D's order: no schedule of these updates is shorter.
Printed, per window:
  - per_launch = sum_k max_e L[e, k]: what K launches that each wait for their deepest env pay;
  - pipelined  = max_e sum_k L[e, k]: what a per-env pipeline (env e's step k + 1 starting when its
    own step k ends) would pay; 1 - pipelined / per_launch is the most that removing the launch
    boundary's tail can gain in kernel B;
  - the floor in ms for both (pos_passes = pos_iters, an upper count: islands leave early).

    python tools/chain_floor.py --agents 1024 --envs 2048 --warmup 2 --steps 10     # the C5 window
    python tools/chain_floor.py --agents 256 --envs 4096 --flocks 4 --warmup 5 --steps 20   # C3
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"), os.path.join(REPO, "gym-macm_amd")]


def window_levels(agents, envs, flocks, warmup, steps, seed, spread, threads, policy="random"):
    """[steps, envs, 4] (touching, levels, islands, largest island) of the timed steps; policy "bots":
    the closed loop with the reference's bots.flock (tests/parity.py flock_bot) on the float32 obs."""
    from gym_macm.settings import flockSettings, to_config
    from oracle import OracleFlock
    from parity import flock_bot
    N = agents
    tidx = None if flocks <= 1 else np.asarray([i * flocks // N for i in range(N)], np.int32)
    cfg = to_config(flockSettings(start_spread=spread), N, max(1, flocks), obs_f64=True)
    orc = OracleFlock(cfg, tidx, envs, seed)
    rng = np.random.default_rng(seed + 1)
    out = np.zeros((steps, envs, 4), np.int32)
    obs = orc.observe()[0] if policy == "bots" else None
    for k in range(warmup + steps):
        if k >= warmup:  # the structure the step is about to solve: the state at its start
            out[k - warmup] = orc.levels()
        if policy == "bots":
            obs = orc.step(flock_bot(obs.astype(np.float32).astype(np.float64)), n_threads=threads)["obs"]
        else:
            orc.step(rng.integers(0, 3, size=(envs, N, 3)).astype(np.uint8), n_threads=threads)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=1024)
    ap.add_argument("--envs", type=int, default=2048)
    ap.add_argument("--flocks", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--spread", type=float, default=20.0)
    ap.add_argument("--policy", choices=("random", "bots"), default="random")
    ap.add_argument("--seed", type=int, default=0x6D61636D)
    ap.add_argument("--vel-iters", type=int, default=8)
    ap.add_argument("--pos-iters", type=int, default=3)
    ap.add_argument("--c-vel", type=float, default=208.0, help="cycles per velocity level step (V3 floor)")
    ap.add_argument("--c-pos", type=float, default=0.0, help="cycles per position level step (V14 floor)")
    ap.add_argument("--ghz", type=float, default=2.4, help="shader clock (ubench: 278 cycles = 117 ns)")
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    t0 = time.time()
    lv = window_levels(a.agents, a.envs, a.flocks, a.warmup, a.steps, a.seed, a.spread, a.threads, a.policy)
    L = lv[..., 1].astype(np.int64)  # [K, E]
    per_launch = int(L.max(axis=1).sum())
    pipelined = int(L.sum(axis=0).max())
    c_pos = a.c_pos if a.c_pos > 0 else a.c_vel
    cyc_per_level = (1 + a.vel_iters) * a.c_vel + a.pos_iters * c_pos
    ms = lambda lv_: lv_ * cyc_per_level / (a.ghz * 1e9) * 1e3  # noqa: E731
    deepest = L.max(axis=1)
    res = {
        "config": dict(agents=a.agents, envs=a.envs, flocks=a.flocks, warmup=a.warmup, steps=a.steps, seed=a.seed,
                       spread=a.spread, policy=a.policy),
        "heaviest_envs": [dict(env=int(e), levels_total=int(L[:, e].sum()), touching_mean=float(lv[:, e, 0].mean()),
                               islands_mean=float(lv[:, e, 2].mean()), largest_island_mean=float(lv[:, e, 3].mean()))
                          for e in np.argsort(-L.sum(axis=0))[:8]],
        "levels_total_percentiles": {str(q): float(np.percentile(L.sum(axis=0), q)) for q in (50, 90, 99, 100)},
        "levels_per_step_deepest": deepest.tolist(),
        "levels_per_step_mean": L.mean(axis=1).round(1).tolist(),
        "touching_mean": float(lv[..., 0].mean()), "touching_max": int(lv[..., 0].max()),
        "per_launch_levels": per_launch, "pipelined_levels": pipelined,
        "pipeline_gain_bound": 1.0 - pipelined / per_launch if per_launch else 0.0,
        "same_env_deepest_steps": int(np.sum(L.argmax(axis=1) == np.bincount(L.argmax(axis=1)).argmax())),
        "cycles_per_level": cyc_per_level, "c_vel": a.c_vel, "c_pos": c_pos, "ghz": a.ghz,
        "chain_floor_ms_per_step": ms(per_launch) / a.steps,
        "chain_floor_ms_per_step_pipelined": ms(pipelined) / a.steps,
        "oracle_seconds": time.time() - t0,
        "note": "actions: numpy default_rng(seed + 1) uniform discrete (not the bench's device draw); "
                "levels from the oracle's state at each step's start; position passes counted as pos_iters",
    }
    s = json.dumps(res, indent=1)
    print(s)
    if a.json:
        with open(a.json, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
