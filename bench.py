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
# The Gauss-Seidel chain floor (roofline.chain_floor_ms): cycles of one velocity / position level step's
# dependent VALU chain, one wave alone on its SIMD (tools/ubench_level.hip V3 / V14 on the MI355X,
# profiles/r05/ubench/), and the shader clock those cycles run at (V0: 278.1 cycles = 117.1 ns)
C_VEL_LEVEL, C_POS_LEVEL, SHADER_GHZ = 208.0, 236.5, 2.375
# the same chains on packed (x, y) pairs (V5 / V16, profiles/r05/ubench/): the form kernel B, the spill
# step and the wave kernel's wide levels run; roofline.chain_frac_packed prices against these
C_VEL_LEVEL_PK, C_POS_LEVEL_PK = 155.4, 224.1
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
SCALAR_SWEEP_MIN_ENVS = 2048  # = kScalarSweepMinEnvs in gym-macm_amd/csrc/flock_step_w64.hip


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _loaded_hip_runtime():
    """The HIP runtime torch already loaded into this process, opened with RTLD_NOLOAD so that no
    second copy is ever loaded (a hard-coded soname could load one, and device flags
    set on it would not reach torch's). Found in /proc/self/maps; refuses if none is loaded."""
    import ctypes
    paths = []
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and os.path.basename(parts[-1]).startswith("libamdhip64.so"):
                paths.append(parts[-1])
    for p in dict.fromkeys(paths):
        try:
            return ctypes.CDLL(p, mode=os.RTLD_NOLOAD | ctypes.RTLD_GLOBAL)
        except OSError:
            continue
    raise SystemExit("--host-wait spin: no HIP runtime (libamdhip64) is loaded in this process")


def _cpu_window(step_fn, acts, warmup, steps, budget_s):
    """Run `warmup` untimed steps, then time up to `steps` steps (the GPU leg's window),
    fewer if they would exceed the budget. Returns (timed steps, seconds, warmup run)."""
    t0 = time.perf_counter()
    step_fn(acts[0])
    per_step = time.perf_counter() - t0
    w_run = 1
    for s in range(1, warmup):
        if (s + 1) * per_step > budget_s:  # warm-up alone would exceed the budget
            break
        step_fn(acts[s % len(acts)])
        w_run += 1
    n = int(max(3, min(steps, budget_s / max(per_step, 1e-6))))
    t0 = time.perf_counter()
    for s in range(n):
        step_fn(acts[(w_run + s) % len(acts)])
    return n, time.perf_counter() - t0, w_run


def cpu_baseline(n_agents, seed, budget_s=15.0, n_envs=4096, warmup=5, steps=20, n_targets=1, tidx=None,
                 acts_host=None, levels_budget_s=0.0):
    """Time the CPU oracle on this host (OpenMP over envs) on the same workload as the GPU
    leg: the same E envs x N agents from reset, `warmup` untimed steps, then the GPU leg's
    `steps` timed (fewer if they would exceed the budget). acts_host: the GPU leg's own actions
    [warmup + steps, E, N, 3] (else uniform draws of the same distribution).
    levels_budget_s > 0: then an untimed replay of the same window records each timed step's
    Gauss-Seidel level structure per env (OracleFlock.levels, for the chain floor); returns
    (baseline dict, levels [steps', E] or None)."""
    from oracle import OracleFlock
    from gym_macm.settings import flockSettings, to_config

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    E = n_envs
    cfg = to_config(flockSettings(), n_agents, n_targets, obs_f64=True)
    orc = OracleFlock(cfg, tidx, E, seed)
    rng = np.random.default_rng(seed + 1)
    bufs = dict(obs=np.zeros((E, n_agents, 4), np.float64), nbr_id=np.zeros((E, n_agents), np.int32),
                reward=np.zeros((E, n_agents), np.float64))
    same = acts_host is not None
    acts = (list(acts_host) if same else
            [rng.integers(0, 3, size=(E, n_agents, 3)).astype(np.uint8) for _ in range(16)])
    n, dt, w_run = _cpu_window(lambda a: orc.step_raw(a, bufs, threads), acts, warmup, steps, budget_s)
    base = dict(value=E * n_agents * n / dt, unit="agent·steps/s", cores=threads, kind="port",
                sample=f"oracle/ C restatement, {E} envs x {n_agents} agents, steps {w_run + 1}..{w_run + n} from "
                       f"reset (the GPU leg times steps {warmup + 1}..{warmup + steps}), "
                       + ("the GPU leg's own actions" if same else "uniform random discrete actions")
                       + f", OpenMP {threads} threads, {dt:.2f} s timed")
    lv = None
    if same and levels_budget_s > 0 and w_run == warmup:
        # untimed replay of the GPU leg's window: the level structure each timed step solves (the first
        # steps of the window when the budget ends earlier: chain_floor records steps_sampled)
        orc2 = OracleFlock(cfg, tidx, E, seed)
        t0 = time.perf_counter()
        rows = []
        for k in range(warmup + steps):
            if k >= warmup:
                rows.append(orc2.levels()[:, 1].copy())
                if time.perf_counter() - t0 > levels_budget_s:
                    break
            orc2.step_raw(acts[k], bufs, threads)
        lv = np.stack(rows) if rows else None
    return base, lv


def chain_floor(levels, rollout, vel_iters=8, pos_iters=3, c_vel=C_VEL_LEVEL, c_pos=C_POS_LEVEL):
    """The Gauss-Seidel chain floor of the timed window, per step: every velocity and position pass
    steps each level of an env's island order once ((1 + vel_iters) x C_VEL_LEVEL + pos_iters x
    C_POS_LEVEL cycles per level, the dependent VALU floors of one wave alone on its SIMD), and a
    launch ends with its deepest env: per step-launch sum_k max_e L[k, e]; one rollout launch of the
    K steps, max_e sum_k L[k, e] (each env's wave runs its steps back to back). Returns (ms per step,
    detail)."""
    L = np.asarray(levels, np.int64)
    K = L.shape[0]
    per_launch, pipelined = int(L.max(axis=1).sum()), int(L.sum(axis=0).max())
    lv = pipelined if rollout else per_launch
    cyc = (1 + vel_iters) * c_vel + pos_iters * c_pos
    ms = lv * cyc / (SHADER_GHZ * 1e9) * 1e3 / K
    return ms, {"levels_per_step_deepest": [int(x) for x in L.max(axis=1)], "levels_mean": float(L.mean()),
                "sum_k_max_e": per_launch, "max_e_sum_k": pipelined, "steps_sampled": K,
                "cycles_per_level": cyc, "c_vel": c_vel, "c_pos": c_pos, "ghz": SHADER_GHZ}


def b_alg_tdm(n_agents, obs_f64=False):
    """Algorithmic bytes per TDM agent-step: state r+w 2 x 40 (as Flock), action 4,
    health/cd_atk/cd_mov f64 + alive u8 r+w 2 x 25, obs (N-1) x 16 (float64: x 32), mask N-1,
    health/alive outputs 9."""
    return 80 + 4 + 50 + (n_agents - 1) * (32 if obs_f64 else 16) + (n_agents - 1) + 9


def cpu_baseline_tdm(team_sizes, seed, budget_s=15.0, n_envs=4096, warmup=5, steps=20):
    """Time the CPU TDM oracle (oracle/tdm_oracle.c, OpenMP over envs) on the GPU leg's window
    (same E envs from reset, `warmup` untimed steps, then up to `steps` timed)."""
    from oracle import OracleTDM
    from gym_macm.tdm_world import tdm_config

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    E = n_envs
    N = sum(team_sizes)
    orc = OracleTDM(tdm_config(team_sizes, obs_f64=True), E, seed)
    rng = np.random.default_rng(seed + 1)
    acts = [tdm_random_actions_np(rng, E, N) for _ in range(16)]
    n, dt, w_run = _cpu_window(lambda a: orc.step(a, threads), acts, warmup, steps, budget_s)
    return dict(value=E * N * n / dt, unit="agent·steps/s", cores=threads, kind="port",
                sample=f"oracle/ C restatement of TDM, {E} envs x {N} agents, steps {w_run + 1}..{w_run + n} from "
                       f"reset (the GPU leg times steps {warmup + 1}..{warmup + steps}), uniform random actions "
                       f"(attack p=0.5), OpenMP {threads} threads, {dt:.2f} s timed")


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


def lib_sha256():
    """sha256 of the HIP library this process loaded (gym_macm._abi.LIB_PATH): a PMC summary is
    quoted as `traffic` only when it was measured on this very binary."""
    import hashlib
    from gym_macm import _abi
    with open(_abi.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch_ranks(n):
    """`--gpus N > 1` without a launcher: start torch.distributed.run with N ranks (this script, the same
    arguments) as a CHILD process and return its exit code. Called before anything touches the GPU; the
    parent never initialises the device and never re-execs itself. The child's stdout is this process's
    (rank 0's JSON line goes straight through)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"--gpus {n} without a launcher: starting {n} ranks under torch.distributed.run")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def dry_run(args, rank, world):
    """--dry-run (test hook, no device work): the launch, the process group, the shard split and the
    counter all-reduce of a real run; every rank contributes its env count. Rank 0 prints the line with
    value null. Lets the CPU suite check that `--gpus N` yields N ranks and N shards."""
    from gym_macm import dist as gdist
    strong = args.total_envs > 0
    if strong:
        e_off, E = gdist.strong_split(args.total_envs, world, rank)
        shards = [list(gdist.strong_split(args.total_envs, world, r)) for r in range(world)]
    else:
        E = args.envs
        e_off = gdist.env_offset(rank, E)
        shards = [[gdist.env_offset(r, E), E] for r in range(world)]
    envs = int(gdist.reduce_counters([E])[0])
    ranks = int(gdist.reduce_counters([1])[0])
    if rank == 0:
        print(json.dumps({"metric": "dry run", "value": None, "n_gpus": world, "ranks_reporting": ranks,
                          "dry_run": True, "config": {"envs_per_gpu": E, "total_envs": envs, "shards": shards,
                                                      "first_env": e_off}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: the launcher's WORLD_SIZE, else 1. N > 1 without a "
                         "launcher starts torch.distributed.run with N ranks as a child process")
    ap.add_argument("--dry-run", action="store_true",
                    help="test hook: launch, process group, shards and the counter all-reduce only (no GPU)")
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
    ap.add_argument("--obs-f64", action="store_true",
                    help="float64 observations (the reference's own width, mvmnt.py:197-220); default float32")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="N > 1: nccl (= RCCL over xGMI, one GPU per rank); gloo: host-side counters, ranks "
                         "may share a GPU (multi-process test of the sharded path on a 1-GPU box)")
    ap.add_argument("--launch", choices=("rollout", "step"), default="rollout",
                    help="rollout: the K timed steps in one launch, each env's wave running its steps back to "
                         "back (random: macm_world_rollout over the actions drawn in advance; bots: "
                         "macm_world_rollout_bots, the bot acting inside the launch; N <= 64, the workgroup path "
                         "launches per step either way); step: one launch per step (plus the bot's). A rollout run "
                         "also times the per-step launches on the same window (per_step_launch)")
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--total-envs", type=int, default=0,
                    help="strong scaling: split this many envs over the ranks (contiguous global env ids, "
                         "BASELINE config 4: 4096 over 8, config 5: 16384 over 8) instead of --envs per GPU; "
                         "actions are drawn for the whole job, so every env's results are those of a "
                         "single-process run")
    ap.add_argument("--outputs", choices=("trajectory", "overwrite"), default="trajectory",
                    help="random policy, rollout launch: trajectory (default) keeps every step's outputs in "
                         "[K, E, N, ...] buffers (macm_world_rollout_traj / macm_tdm_rollout_traj), as the reference "
                         "returns (obs, rewards) from every env.step (mvmnt.py:140); overwrite: every step "
                         "overwrites one output set, the caller receives only the last step's "
                         "(macm_world_rollout / macm_tdm_rollout)")
    ap.add_argument("--trajectory", action="store_true", help="= --outputs trajectory (kept for old scripts)")
    ap.add_argument("--host-wait", choices=("default", "spin"), default="default",
                    help="spin: hipSetDeviceFlags(hipDeviceScheduleSpin) before the device is initialised, so "
                         "the host polls for completion instead of waiting for an interrupt (A/B of the host "
                         "gap around the timed launch)")
    ap.add_argument("--dump-final", default=None,
                    help="test hook: every rank writes its final state and counters to PATH.rank<r>.npz")
    args = ap.parse_args()
    # --gpus against the launcher, before any GPU call: the driver's scaling leg may
    # run `python bench.py --gpus N` (no launcher) or `torchrun --nproc-per-node N bench.py --gpus N`
    launcher = "WORLD_SIZE" in os.environ or "MASTER_ADDR" in os.environ
    if args.gpus is not None and args.gpus < 1:
        raise SystemExit(f"--gpus {args.gpus}: need at least one rank")
    if not launcher and (args.gpus or 1) > 1:
        sys.exit(_launch_ranks(args.gpus))
    if launcher and args.gpus is not None and int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE="
                         f"{os.environ.get('WORLD_SIZE', '1')} ranks: they must agree")
    if args.traffic_json is None:
        args.traffic_json = os.path.join(REPO, "profiles", "pmc_flock_step.json" if args.env == "flock"
                                         else "pmc_tdm_step.json")

    if args.host_wait == "spin":
        hip = _loaded_hip_runtime()
        rc = hip.hipSetDeviceFlags(1)  # hipDeviceScheduleSpin
        if rc != 0:
            raise SystemExit(f"hipSetDeviceFlags(hipDeviceScheduleSpin) failed: {rc}")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # a launcher (torchrun) sets MASTER_ADDR: the process group exists then even for one rank, so
    # `torchrun --nproc-per-node 1` runs the RCCL branch (init, barriers, device all-reduces) on a
    # one-GPU box; a plain `python bench.py` (the driver's N=1 run) has no process group
    launched = world > 1 or "MASTER_ADDR" in os.environ
    if args.dry_run:
        if launched:
            dist.init_process_group("gloo")
        dry_run(args, rank, world)
        if launched:
            dist.destroy_process_group()
        return
    if launched and args.dist_backend == "nccl":
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif launched:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    red_dev = dev if args.dist_backend == "nccl" else None  # gloo reduces host tensors

    from gym_macm import dist as gdist

    K, W = args.steps, args.warmup
    strong = args.total_envs > 0
    if strong and args.total_envs < world:
        # a rank with no env could not create a world and the others would wait at the first barrier
        raise SystemExit(f"--total-envs {args.total_envs} < {world} ranks: every rank needs at least one env")
    if strong:  # this rank's contiguous share of the job's envs
        e_off, E = gdist.strong_split(args.total_envs, world, rank)
    else:  # weak: --envs per GPU
        E = args.envs
        e_off = gdist.env_offset(rank, E)
    if args.trajectory:
        args.outputs = "trajectory"
    # every step's outputs are what env.step returns; the forms that get them without a trajectory
    # buffer are the closed loop (the bot consumes each step's obs inside the launch) and one launch
    # per step (the caller reads each step's outputs between launches)
    use_traj = args.outputs == "trajectory" and args.policy == "random" and args.launch == "rollout"
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + 1 + (0 if strong else rank))

    # strong: every rank draws the whole job's actions and keeps its rows, so each env sees the same
    # actions at any rank count; that is (W + K) x total_envs x N x A bytes per rank (BASELINE C5,
    # 16,384 x 1024 agents x 3 B, 12 steps: 0.6 GB), freed once the rank's slice is copied
    def draw(shape, high=3):  # uniform uint8 in [0, high); strong: the whole job's draw, this rank's rows
        if not strong:
            return torch.randint(0, high, shape, dtype=torch.uint8, device=dev, generator=gen)
        full = torch.randint(0, high, (shape[0], args.total_envs) + tuple(shape[2:]), dtype=torch.uint8, device=dev,
                             generator=gen)
        return full[:, e_off:e_off + E].contiguous()
    if args.env == "flock":
        from gym_macm.vec import FlockVec
        N = args.agents
        targets = None if args.flocks <= 1 else [i * args.flocks // N for i in range(N)]
        vec = FlockVec(E, n_agents=[N], targets=targets, seed=args.seed, env_offset=e_off,
                       device=dev, obs_dtype=torch.float64 if args.obs_f64 else torch.float32)
        world_h = vec.world
        acts = draw((W + K, E, N, 3))
        stride = E * N * 3
    else:
        from gym_macm.tdm_world import TdmWorld, tdm_config
        teams = [int(x) for x in args.teams.split(",")]
        N = sum(teams)
        world_h = TdmWorld(tdm_config(teams, obs_f64=args.obs_f64), E, device=dev)
        world_h.reset(args.seed, e_off)
        acts = draw((W + K, E, N, 4))
        acts[..., 3] = draw((W + K, E, N), 2)
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
    rollout = args.launch == "rollout"
    traj = world_h.trajectory_buffers(K) if use_traj else None
    if args.env == "tdm":  # the tail observation's snapshots for the longer of the two rollouts, ahead
        world_h.reserve(max(W, K))
    traj_out = world_h.traj_outputs(traj) if use_traj else None  # the C-ABI struct, built outside the timing
    rname = ("macm_world_rollout" if args.env == "flock" else "macm_tdm_rollout") + ("_traj" if traj is not None else "")
    log(f"rank {rank}/{world}: {E} envs x {N} agents, warmup {W}, timed {K}, "
        f"{'one rollout launch' if rollout else 'one launch per step'}")

    def timed_window(roll):
        """W untimed warm-up steps from the current state, then K timed steps (bracketed by a barrier
        and synchronisations); returns (host seconds, event ms on the launch stream)."""
        if roll and args.policy == "bots":  # closed loop in one launch: the bot acts inside it
            if W:
                world_h.rollout_bots_raw(loop_ptr, W, sh)
        elif roll:
            if W:
                world_h.rollout_raw(base, W, sh)
        else:
            for w in range(W):
                step(base + w * stride, sh)
        torch.cuda.synchronize(dev)
        if args.env == "flock":
            world_h.reset_counters()  # and the reward sums
        spilled0 = world_h.spilled()
        # the events are created (lazily, at their first record) before the timed region
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        ev1.record(stream)
        if launched:
            dist.barrier()
        # the timed launch with its ctypes arguments converted up front (Python work ahead of the launch)
        go = None
        if roll and traj is not None and args.policy != "bots":
            go = world_h.rollout_traj_launcher(base + W * stride, K, traj_out, sh)
        torch.cuda.synchronize(dev)
        ev0.record(stream)  # on the idle stream: its timestamp falls just before t0
        t0 = time.perf_counter()
        if roll and args.policy == "bots":
            world_h.rollout_bots_raw(loop_ptr, K, sh)
        elif roll and traj is not None:
            go()
        elif roll:
            world_h.rollout_raw(base + W * stride, K, sh)
        else:
            for k in range(K):
                step(base + (W + k) * stride, sh)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        if launched:
            dist.barrier()
        return t1 - t0, ev0.elapsed_time(ev1), world_h.spilled() - spilled0

    elapsed, ev_ms, spilled = timed_window(rollout)
    kernel_ms = ev_ms / K  # per step on the launch stream (a rollout launch covers all K steps)
    # one small RCCL all-reduce of counters after the timed region (no data-path collective)
    status = int(gdist.reduce_counters([world_h.status()], device=red_dev, op="max")[0])
    cnt = gdist.reduce_counters(world_h.counters(), device=red_dev)
    spilled = int(gdist.reduce_counters([spilled], device=red_dev)[0])
    # Σreward (float64): every rank's per-env sums gathered and added in global env
    # order, so the total is bit-identical to a single-process run of the job at any rank count
    reward_sum = gdist.reduce_reward_sums(world_h.reward_sums()[0], device=red_dev) if args.env == "flock" else None
    elapsed = gdist.reduce_max(elapsed, device=red_dev)
    total_agent_steps = (args.total_envs if strong else world * E) * N * K
    if args.env == "flock":
        assert int(cnt[0]) == total_agent_steps, (cnt, total_agent_steps)
    if status != 0:
        raise RuntimeError(f"device status bits {status}: a capacity overflowed, results invalid")
    value = total_agent_steps / elapsed
    if args.dump_final:
        st = world_h.get_state()
        np.savez(f"{args.dump_final}.rank{rank}.npz", env_offset=e_off, counters=world_h.counters(),
                 **{k: v for k, v in st.items() if isinstance(v, np.ndarray)})

    if rank == 0:
        # float64 obs: the 4 obs values take 8 B each (Flock +16 B; TDM +16 B per observed agent)
        b_alg = (B_ALG + (16 if args.obs_f64 else 0)) if args.env == "flock" else b_alg_tdm(N, args.obs_f64)
        achieved_gbs = b_alg * E * N / (kernel_ms * 1e-3) / 1e9
        ncap = 32 if N <= 32 else 64
        if args.env == "tdm":
            # N > 64: the workgroup TDM step (tdm_step_wg.hip), one launch per step in either form
            kname = (f"env_{'rollout' if rollout else 'step'}_w64<1, {ncap}, float, false>" if N <= 64
                     else "tdm_step_wg<float>")
            scal = "false"
        else:
            # N > 64: the workgroup path's three launches per step (split step; kernel_ms covers all)
            # N > 32 with >= 2048 envs: the scalar-sweep instantiation (flock_step_w64.hip,
            # kScalarSweepMinEnvs)
            scal = "true" if (ncap == 64 and E >= SCALAR_SWEEP_MIN_ENVS) else "false"
            kname = (f"env_{'rollout' if rollout else 'step'}_w64<0, {ncap}, float, {scal}>" if N <= 64
                     else "flock_step_wg_a + flock_solve_wg + flock_step_wg_c<float>")
        traffic = None
        tj = load_traffic(args.traffic_json)
        if args.obs_f64:  # the scalar sweep exists only in the float32-obs instantiation
            kname = kname.replace("float", "double").replace("double, true>", "double, false>")

        spl = K if (rollout and N <= 64) else 1  # env steps per launch of the priced kernel
        traffic_src = None
        oform = "trajectory" if traj is not None else "overwrite"
        if (tj and tj.get("envs") == E and tj.get("agents") == N and tj.get("kernel") == kname
                and tj.get("policy", "random") == args.policy and tj.get("steps_per_launch", 1) == spl
                and (spl == 1 or args.policy != "random" or tj.get("outputs", "overwrite") == oform)):
            if tj.get("lib_sha256") and tj["lib_sha256"] == lib_sha256():
                # per step (a rollout launch's bytes over its steps), like achieved
                traffic = tj.get("hbm_bytes_per_launch") / tj.get("steps_per_launch", 1)
                traffic_src = f"{os.path.relpath(args.traffic_json, REPO)} (commit {tj.get('commit')})"
            else:
                traffic_src = (f"{os.path.relpath(args.traffic_json, REPO)} was measured on another build "
                               f"(lib sha256 {str(tj.get('lib_sha256'))[:12]}): not quoted")
        hbm_frac = None if traffic is None else traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
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
        # MACM_LAUNCH_SPLIT_OBS: every TDM step / rollout but the closed-loop rollout (its bot reads each
        # step's observation inside the launch)
        lflags = world_h.launch_flags() if args.env == "tdm" else 0
        split = (args.env == "tdm" and N <= 64 and bool(lflags & 2)
                 and not (rollout and args.policy == "bots"))
        # MACM_LAUNCH_TAIL_OBS: the trajectory rollout observes in the tail of its own launch (TailObs)
        tail = (args.env == "tdm" and N <= 64 and bool(lflags & 4) and rollout and traj is not None
                and args.policy == "random")
        if tail:
            split = False
        slices = world_h.rollout_slices() if (args.env == "flock" and N > 64) else 0
        if split:  # TDM below 1024 envs: pose snapshots, the observation in a kernel of its own
            kname += " + tdm_observe_snap<" + ("double" if args.obs_f64 else "float") + ">"
        if tail:
            kname += " (tail observation)"
        if rollout and N <= 64:
            if tail:
                launch_desc = (f"one {rname} launch for the K timed steps: each env's wave steps its K steps writing "
                               "pose snapshots, then the finished waves and one observe-only wave per env observe "
                               "the (step, env) rows beside the remaining envs' physics")
            elif split and traj is not None:
                launch_desc = (f"{rname}: the K timed steps in rollout launches of 8 steps that write pose "
                               "snapshots, each chunk's observation (tdm_observe_snap) on a second stream beside "
                               "the next chunk's physics")
            elif split:
                launch_desc = f"one {rname} launch for the K timed steps, the last step's observation by tdm_observe_snap"
            else:
                launch_desc = f"one {rname}{'_bots' if args.policy == 'bots' else ''} launch for the K timed steps"
        elif not rollout:
            launch_desc = "one step per launch" + (" (+ tdm_observe_snap)" if split else "")
        elif slices:
            launch_desc = (f"{rname}, workgroup path: {slices} env slices on streams of their own, 3 launches per "
                           "step each, no join between steps")
        else:
            launch_desc = f"{rname}, workgroup path: 3 launches per step"
        out = {
            "metric": metric,
            "value": value,
            "unit": "agent·steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",  # the physics; observations per config.obs
            "data": "synthetic",
            "config": {
                "workload": workload,
                "envs_per_gpu": E, "n_agents": N,
                "total_envs": args.total_envs if strong else E * world,
                "split": (f"strong: {args.total_envs} envs over {world} ranks (this rank: global envs "
                          f"{e_off}..{e_off + E - 1})") if strong else f"weak: {E} envs per GPU",
                # every rank's contiguous shard [first global env id, env count]: the counters above
                # are their all-reduced totals
                "shards": ([list(gdist.strong_split(args.total_envs, world, r)) for r in range(world)] if strong
                           else [[gdist.env_offset(r, E), E] for r in range(world)]),
                "parallelism": f"env-sharded x{world} (no data-path collective)"
                               + ("" if not launched else ", RCCL counters" if args.dist_backend == "nccl"
                                  else ", gloo counters (test mode)"),
                "obs": "float64" if args.obs_f64 else "float32",
                # per-env contact-list capacity and spill working-set slots (macm_world_create's
                # defaults from 1/8 of the device's free memory)
                "max_contacts": int(world_h.C) if args.env == "flock" else None,
                "spill_slots": int(world_h.spill_slots) if args.env == "flock" else None,
                "launch": launch_desc,
                # what the caller gets back: the reference returns (obs, rewards) from every env.step
                # (mvmnt.py:140); the plain rollout launch overwrites its outputs every step
                "outputs": ("every step's ([K, E, N, ...] trajectory buffers)" if traj is not None
                            else "every step's (one launch per step)" if not rollout
                            else "every step's obs consumed by the device bot inside the launch; the caller "
                                 "receives the last step's" if args.policy == "bots"
                            else "overwrite: the last step's (each step overwrites them; counters cover all K "
                                 "steps)"),
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                # the PMC-measured HBM bytes over the same time: how far from HBM-bound the kernel is
                "hbm_frac_measured": hbm_frac,
                "traffic_source": traffic_src,
                "kernel": kname, "kernel_ms": kernel_ms,  # per step
                "steps_per_launch": spl,
                "bytes_alg_per_step": b_alg * E * N,
                "bytes_alg_per_launch": b_alg * E * N * spl,
            },
            # env-steps taken by the spill step (dense envs past the fast kernels' LDS capacities) in
            # the timed window: capacities follow the box's free memory (macm_world_create)
            "spilled_env_steps": spilled,
        }
        if args.env == "flock":
            out["counters"] = {"agent_steps": int(cnt[0]), "collided_agent_steps": int(cnt[1]),
                               "positive_reward_agent_steps": int(cnt[2]), "done_env_steps": int(cnt[3]),
                               "reward_sum": reward_sum}
        else:
            out["counters"] = {"alive_agent_steps": int(cnt[0]), "melee_attacks": int(cnt[1]),
                               "deaths": int(cnt[2]), "done_env_steps": int(cnt[3])}
        if rollout and world == 1:
            # the same window again with one launch per step (what a closed-loop policy needs)
            if args.env == "flock":
                vec.reset()
            else:
                world_h.reset(args.seed, e_off)
            if args.policy == "bots":
                policy()  # the first actions from the initial obs again
            el2, ev2, _ = timed_window(False)
            out["per_step_launch"] = {"value": E * N * K / el2, "ms_per_step": el2 / K * 1e3,
                                      "kernel_ms_per_step": ev2 / K}
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline (oracle) ...")
            if args.env == "flock":
                # the GPU leg's own actions when the window is short (the driver's 25 steps)
                ah = acts.cpu().numpy() if (args.policy == "random" and W + K <= 64) else None
                out["cpu_baseline"], lv = cpu_baseline(
                    N, args.seed, args.cpu_budget, E, W, K, n_targets=args.flocks if args.flocks > 1 else 1,
                    tidx=None if targets is None else np.asarray(targets, np.int32), acts_host=ah,
                    levels_budget_s=args.cpu_budget)
                if lv is not None:
                    fl_ms, fl = chain_floor(lv, rollout and N <= 64)
                    out["roofline"]["chain_floor_ms"] = fl_ms
                    out["roofline"]["chain_frac"] = fl_ms / kernel_ms
                    out["roofline"]["chain_floor"] = fl
                    fp_ms, _ = chain_floor(lv, rollout and N <= 64, c_vel=C_VEL_LEVEL_PK, c_pos=C_POS_LEVEL_PK)
                    out["roofline"]["chain_floor_packed_ms"] = fp_ms
                    out["roofline"]["chain_frac_packed"] = fp_ms / kernel_ms
            else:
                out["cpu_baseline"] = cpu_baseline_tdm(teams, args.seed, args.cpu_budget, E, W, K)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if launched:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
