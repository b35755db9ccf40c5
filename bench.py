"""bench.py — agent·steps/sec of the cm-flock-v0 step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One "step" = one env.step of every env on this rank: one HIP launch of
env_step_w64 over E envs x N agents (physics + rewards + observations; N > 64: the
workgroup path's three launches), with
the actions pre-generated on the device (uniform {0,1,2}^3 uint8, the
MultiDiscrete([3,3,3]) action space) and outputs written to device tensors.
Weak scaling: every rank runs its own E envs (global env ids rank*E .. rank*E+E-1),
no collective on the data path; one all-reduce of counters after the timed region.

Rank 0 prints ONE JSON line. `roofline` prices the step kernel against HBM with the
algorithmic bytes of SURVEY.md §8(d) (B_alg = 107 B per agent-step); `cpu_baseline`
times the CPU oracle (oracle/, a C restatement of the reference's path) on this
host's cores over a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gym-macm_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

B_ALG = 107  # bytes per agent-step: state r+w 2x40, action 3, obs 20, reward 4
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
SCALAR_SWEEP_MIN_ENVS = 2048  # = kScalarSweepMinEnvs in gym-macm_amd/csrc/flock_step_w64.hip


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(n_agents, seed, budget_s=15.0, n_envs=4096):
    """Time the CPU oracle on this host (OpenMP over envs) on a bounded sample of the
    same workload: the same E envs x N agents, as many steps as fit the budget."""
    from oracle import OracleFlock
    from gym_macm.settings import flockSettings, to_config

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    E = n_envs
    cfg = to_config(flockSettings(), n_agents, 1, obs_f64=True)
    orc = OracleFlock(cfg, None, E, seed)
    rng = np.random.default_rng(seed + 1)
    bufs = dict(obs=np.zeros((E, n_agents, 4), np.float64), nbr_id=np.zeros((E, n_agents), np.int32),
                reward=np.zeros((E, n_agents), np.float64))
    pre = [rng.integers(0, 3, size=(E, n_agents, 3)).astype(np.uint8) for _ in range(8)]
    t0 = time.perf_counter()
    for a in pre[:3]:
        orc.step_raw(a, bufs, threads)
    per_step = (time.perf_counter() - t0) / 3
    steps = int(max(5, budget_s / max(per_step, 1e-6)))
    acts = [rng.integers(0, 3, size=(E, n_agents, 3)).astype(np.uint8) for _ in range(16)]
    t0 = time.perf_counter()
    for s in range(steps):
        orc.step_raw(acts[s % 16], bufs, threads)
    dt = time.perf_counter() - t0
    return dict(value=E * n_agents * steps / dt, unit="agent·steps/s", cores=threads, kind="port",
                sample=f"oracle/ C restatement, {E} envs x {n_agents} agents x {steps} steps (after 3 "
                       f"warm-up steps) from reset, uniform random discrete actions, OpenMP {threads} threads, "
                       f"{dt:.1f} s")


def b_alg_tdm(n_agents):
    """Algorithmic bytes per TDM agent-step (float32 obs): state r+w 2 x 40 (as Flock),
    action 4, health/cd_atk/cd_mov f64 + alive u8 r+w 2 x 25, obs (N-1) x 16, mask N-1,
    health/alive outputs 9."""
    return 80 + 4 + 50 + (n_agents - 1) * 16 + (n_agents - 1) + 9


def cpu_baseline_tdm(team_sizes, seed, budget_s=15.0, n_envs=4096):
    """Time the CPU TDM oracle (oracle/tdm_oracle.c, OpenMP over envs) on a bounded
    sample of the same workload (same E envs, as many steps as fit the budget)."""
    from oracle import OracleTDM
    from gym_macm.tdm_world import tdm_config

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    E = n_envs
    N = sum(team_sizes)
    orc = OracleTDM(tdm_config(team_sizes, obs_f64=True), E, seed)
    rng = np.random.default_rng(seed + 1)
    acts = [tdm_random_actions_np(rng, E, N) for _ in range(16)]
    t0 = time.perf_counter()
    for a in acts[:3]:
        orc.step(a, threads)
    per_step = (time.perf_counter() - t0) / 3
    steps = int(max(5, budget_s / max(per_step, 1e-6)))
    t0 = time.perf_counter()
    for s in range(steps):
        orc.step(acts[s % 16], threads)
    dt = time.perf_counter() - t0
    return dict(value=E * N * steps / dt, unit="agent·steps/s", cores=threads, kind="port",
                sample=f"oracle/ C restatement of TDM, {E} envs x {N} agents x {steps} steps (after 3 warm-up "
                       f"steps) from reset, uniform random actions (attack p=0.5), OpenMP {threads} threads, "
                       f"{dt:.1f} s")


def tdm_random_actions_np(rng, E, N):
    a = rng.integers(0, 3, size=(E, N, 4)).astype(np.uint8)
    a[..., 3] = rng.integers(0, 2, size=(E, N))
    return a


def load_traffic(path):
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        j = json.load(f)
    return j


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--agents", type=int, default=64)
    ap.add_argument("--flocks", type=int, default=1, help="targets = i // (agents / flocks) (config 3: 4)")
    ap.add_argument("--seed", type=int, default=0x6D61636D)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--env", choices=("flock", "tdm"), default="flock",
                    help="flock: cm-flock-v0 (the metric); tdm: cm-tdm-v0 (config 4, --teams)")
    ap.add_argument("--teams", default="16,16", help="TDM team sizes (config 4: 16,16)")
    ap.add_argument("--policy", choices=("random", "bots"), default="random",
                    help="random: pre-generated uniform actions (the metric); bots: closed loop with the "
                         "device bots.flock / bots.combat kernels inside the timed region")
    ap.add_argument("--traffic-json", default=None)
    args = ap.parse_args()
    if args.traffic_json is None:
        args.traffic_json = os.path.join(REPO, "profiles", "pmc_flock_step.json" if args.env == "flock"
                                         else "pmc_tdm_step.json")

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from gym_macm import dist as gdist

    E, K, W = args.envs, args.steps, args.warmup
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + 1 + rank)
    if args.env == "flock":
        from gym_macm.vec import FlockVec
        N = args.agents
        targets = None if args.flocks <= 1 else [i * args.flocks // N for i in range(N)]
        vec = FlockVec(E, n_agents=[N], targets=targets, seed=args.seed, env_offset=gdist.env_offset(rank, E),
                       device=dev)
        world_h = vec.world
        acts = torch.randint(0, 3, (W + K, E, N, 3), dtype=torch.uint8, device=dev, generator=gen)
        stride = E * N * 3
    else:
        from gym_macm.tdm_world import TdmWorld, tdm_config
        teams = [int(x) for x in args.teams.split(",")]
        N = sum(teams)
        world_h = TdmWorld(tdm_config(teams), E, device=dev)
        world_h.reset(args.seed, gdist.env_offset(rank, E))
        acts = torch.randint(0, 3, (W + K, E, N, 4), dtype=torch.uint8, device=dev, generator=gen)
        acts[..., 3] = torch.randint(0, 2, (W + K, E, N), dtype=torch.uint8, device=dev, generator=gen)
        stride = E * N * 4
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    step = world_h.step_raw
    base = acts.data_ptr()
    if args.policy == "bots":
        # closed loop: every step reads the actions the previous step's bot kernel wrote
        from gym_macm import bots
        a_loop = acts[0].clone()
        if args.env == "flock":
            def policy():
                bots.flock_actions(world_h.obs, out=a_loop)
        else:
            def policy():
                bots.combat_actions(world_h.obs, world_h.mask, out=a_loop)
        loop_ptr = a_loop.data_ptr()
        policy()

        def step(_ptr, sh_):  # noqa: F811
            world_h.step_raw(loop_ptr, sh_)
            policy()
    log(f"rank {rank}/{world}: {E} envs x {N} agents, warmup {W}, timed {K}")
    for w in range(W):
        step(base + w * stride, sh)
    torch.cuda.synchronize(dev)
    if args.env == "flock":
        world_h.reset_counters()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(K):
        step(base + (W + k) * stride, sh)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    kernel_ms = ev0.elapsed_time(ev1) / K  # per launch, on the launch stream
    # one small RCCL all-reduce of counters after the timed region (no data-path collective)
    status = int(gdist.reduce_counters([world_h.status()], device=dev, op="max")[0])
    cnt = gdist.reduce_counters(world_h.counters(), device=dev)
    elapsed = gdist.reduce_max(elapsed, device=dev)
    total_agent_steps = world * E * N * K
    if args.env == "flock":
        assert int(cnt[0]) == total_agent_steps, (cnt, total_agent_steps)
    if status != 0:
        raise RuntimeError(f"device status bits {status}: a capacity overflowed, results invalid")
    value = total_agent_steps / elapsed

    if rank == 0:
        b_alg = B_ALG if args.env == "flock" else b_alg_tdm(N)
        achieved_gbs = b_alg * E * N / (kernel_ms * 1e-3) / 1e9
        ncap = 32 if N <= 32 else 64
        if args.env == "tdm":
            kname = f"env_step_w64<1, {ncap}, float, false>"
        else:
            # N > 64: the workgroup path's three launches per step (split step; kernel_ms covers all)
            # N > 32 with >= 2048 envs: the scalar-sweep instantiation (flock_step_w64.hip,
            # kScalarSweepMinEnvs)
            scal = "true" if (ncap == 64 and E >= SCALAR_SWEEP_MIN_ENVS) else "false"
            kname = (f"env_step_w64<0, {ncap}, float, {scal}>" if N <= 64
                     else "flock_step_wg_a + flock_solve_wg + flock_step_wg_c<float>")
        traffic = None
        tj = load_traffic(args.traffic_json)
        if (tj and tj.get("envs") == E and tj.get("agents") == N and tj.get("kernel") == kname
                and tj.get("policy", "random") == args.policy):
            traffic = tj.get("hbm_bytes_per_launch")
        with open(os.path.join(REPO, "BASELINE.json")) as f:
            metric = json.load(f)["metric"]
        if args.env == "tdm":
            metric = "agent·steps/sec, cm-tdm-v0 (config 4)"
            workload = (f"cm-tdm-v0 n_agents={teams} x {E} envs per GPU, " + (
                "uniform random actions (MultiDiscrete[3,3,3,2]) pre-generated on device" if args.policy == "random"
                else "closed loop with the device bots.combat kernel (timed)") +
                f", from reset (seed {args.seed:#x}); agent-steps count every agent slot")
        else:
            workload = (f"cm-flock-v0 n_agents=[{N}]{f' targets=i//{N // args.flocks}' if args.flocks > 1 else ''} "
                        f"x {E} envs per GPU, " + (
                            "uniform random discrete actions (MultiDiscrete[3,3,3]) pre-generated on device"
                            if args.policy == "random" else "closed loop with the device bots.flock kernel (timed)") +
                        f", from reset (seed {args.seed:#x})")
        out = {
            "metric": metric,
            "value": value,
            "unit": "agent·steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": workload,
                "envs_per_gpu": E, "n_agents": N, "total_envs": E * world,
                "parallelism": f"env-sharded x{world} (no data-path collective)",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                "kernel": kname, "kernel_ms": kernel_ms,
                "bytes_alg_per_launch": b_alg * E * N,
            },
        }
        if args.env == "flock":
            out["counters"] = {"agent_steps": int(cnt[0]), "collided_agent_steps": int(cnt[1]),
                               "positive_reward_agent_steps": int(cnt[2]), "done_env_steps": int(cnt[3])}
        else:
            out["counters"] = {"alive_agent_steps": int(cnt[0]), "melee_attacks": int(cnt[1]),
                               "deaths": int(cnt[2]), "done_env_steps": int(cnt[3])}
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline (oracle) ...")
            if args.env == "flock":
                out["cpu_baseline"] = cpu_baseline(N, args.seed, args.cpu_budget, E)
            else:
                out["cpu_baseline"] = cpu_baseline_tdm(teams, args.seed, args.cpu_budget, E)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
