"""Thin Python handle over the C-ABI world (include/macm.h), with torch tensors as
device memory and torch's current stream as the launch stream.

This replaces the reference's framework plugin point — ``NoRender(FrameworkBase)``
owning one ``b2World`` per env (gym_macm/backends/no_render.py:4-19,
gym_macm/cm_framework.py:155-167) — with one device-resident world of E envs.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _abi


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def check_traj(traj: dict, spec: dict, K: int, device, keys) -> list:
    """The caller's trajectory buffers in `keys` order (None where absent), each checked against
    spec[key] = (dtype, per-step shape) before any kernel writes K rows into it: a buffer of the
    wrong dtype, env count or agent count would be overrun on the device."""
    unknown = set(traj) - set(spec)
    if unknown:
        raise ValueError(f"unknown trajectory buffers {sorted(unknown)}; expected a subset of {list(keys)}")
    out = []
    for k in keys:
        t = traj.get(k)
        if t is not None:
            dt, shp = spec[k]
            if (not isinstance(t, torch.Tensor) or t.device != device or not t.is_contiguous() or t.dim() < 1
                    or t.shape[0] < K or t.dtype != dt or tuple(t.shape[1:]) != tuple(shp)):
                got = (f"{tuple(t.shape)} {t.dtype} on {t.device}" if isinstance(t, torch.Tensor) else type(t).__name__)
                raise ValueError(f"trajectory buffer {k!r} must be a contiguous {dt} tensor [>= {K}, "
                                 f"{', '.join(map(str, shp))}] on {device}; got {got}")
        out.append(t)
    return out


class World:
    """E independent envs of one Flock configuration on one GPU.

    Outputs are written into preallocated tensors owned by this object and
    reused by every call (clone them to keep a step's values).
    """

    def __init__(self, cfg: _abi.MacmConfig, targets_idx=None, n_envs: int = 1, device=None,
                 max_contacts: int = 0, host_outputs: bool = False):
        self.L = _abi.lib()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise ValueError("the HIP world lives on a GPU device (no CPU fallback)")
        self.device = device
        self.cfg = cfg
        self.E = int(n_envs)
        self.N = int(cfg.n_agents)
        self.T = int(cfg.n_targets)
        ti = None
        if targets_idx is not None:
            self._tidx = np.ascontiguousarray(np.asarray(targets_idx, np.int32))
            if self._tidx.shape != (self.N,):
                raise ValueError(f"targets_idx must have length n_agents={self.N}")
            ti = self._tidx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            _abi.check(self.L.macm_world_create(ctypes.byref(cfg), ti, self.E, device.index or 0,
                                                int(max_contacts), ctypes.byref(h)), "macm_world_create")
        self.h = h
        info = _abi.MacmWorldInfo()
        _abi.check(self.L.macm_world_info_get(self.h, ctypes.byref(info)), "macm_world_info_get")
        self.info = info
        self.OD = info.obs_dim
        self.C = info.max_contacts
        self.spill_slots = info.spill_slots
        odt = torch.float64 if cfg.obs_f64 else torch.float32
        # host_outputs: outputs live in pinned host memory that the kernels write over
        # the bus (zero-copy views for the small-E dict API; actions may be pinned too)
        self.host_outputs = bool(host_outputs)
        kw = dict(pin_memory=True) if self.host_outputs else dict(device=device)
        self.obs = torch.empty((self.E, self.N, self.OD), dtype=odt, **kw)
        self.nbr_id = torch.empty((self.E, self.N), dtype=torch.int32, **kw)
        self.reward = torch.empty((self.E, self.N), dtype=torch.float32, **kw)
        self.collided = torch.empty((self.E, self.N), dtype=torch.uint8, **kw)
        self.done = torch.zeros((self.E,), dtype=torch.uint8, **kw)
        self._out = _abi.MacmOutputs(_ptr(self.obs), _ptr(self.nbr_id), _ptr(self.reward), _ptr(self.collided),
                                     _ptr(self.done))
        self._out_obs = _abi.MacmOutputs(_ptr(self.obs), _ptr(self.nbr_id), None, None, None)

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.L.macm_world_destroy(h)
            except Exception:
                pass
            self.h = None

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # -- lifecycle ---------------------------------------------------------
    def reset(self, seed: int, env_offset: int = 0):
        """Env e := Flock(...) after random.seed(seed + env_offset + e); writes the initial obs."""
        _abi.check(self.L.macm_world_reset(self.h, int(seed), int(env_offset), ctypes.byref(self._out_obs),
                                           self._stream()), "macm_world_reset")
        self.done.zero_()
        return self.obs, self.nbr_id

    def place(self, pos, angle, targets):
        """Initialise from caller-drawn poses (float32 arrays [E,N,2], [E,N], [E,T,2])."""
        pos = np.ascontiguousarray(pos, np.float32).reshape(self.E, self.N, 2)
        angle = np.ascontiguousarray(angle, np.float32).reshape(self.E, self.N)
        targets = np.ascontiguousarray(targets, np.float32).reshape(self.E, self.T, 2)
        _abi.check(self.L.macm_world_place(self.h, pos.ctypes.data, angle.ctypes.data, targets.ctypes.data,
                                           ctypes.byref(self._out_obs), self._stream()), "macm_world_place")
        self.done.zero_()
        return self.obs, self.nbr_id

    def reset_envs(self, mask=None):
        """New episodes in the envs where `mask` (uint8/bool tensor [E] on this device,
        e.g. ``self.done``; None = all) is set, continuing each env's random stream
        (macm_world_reset_envs). Asynchronous; writes the new initial obs for those envs."""
        ptr = None
        if mask is not None:
            if mask.dtype == torch.bool:
                mask = mask.to(torch.uint8)
            if mask.device != self.device or tuple(mask.shape) != (self.E,) or mask.dtype != torch.uint8:
                raise ValueError(f"mask must be a uint8/bool tensor [{self.E}] on {self.device}")
            ptr = _ptr(mask.contiguous())
        _abi.check(self.L.macm_world_reset_envs(self.h, ptr, ctypes.byref(self._out_obs), self._stream()),
                   "macm_world_reset_envs")
        return self.obs, self.nbr_id

    # -- hot path ------------------------------------------------------------
    def step(self, actions: torch.Tensor):
        """actions: discrete uint8/int8 [E,N,3] or continuous float32 [E,N,2], on this device."""
        pinned_ok = self.host_outputs and actions.device.type == "cpu" and actions.is_pinned()
        if (actions.device != self.device and not pinned_ok) or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous tensor on the world's device (or pinned host "
                             "memory with host_outputs)")
        if self.cfg.action_mode == _abi.ACTION_DISCRETE:
            if actions.dtype not in (torch.uint8, torch.int8) or tuple(actions.shape) != (self.E, self.N, 3):
                raise ValueError(f"discrete actions must be uint8/int8 [{self.E},{self.N},3]")
        else:
            if actions.dtype != torch.float32 or tuple(actions.shape) != (self.E, self.N, 2):
                raise ValueError(f"continuous actions must be float32 [{self.E},{self.N},2]")
        _abi.check(self.L.macm_world_step(self.h, _ptr(actions), ctypes.byref(self._out), self._stream()),
                   "macm_world_step")
        return self.obs, self.nbr_id, self.reward, self.done

    def step_raw(self, actions_ptr: int, stream_handle: int) -> None:
        """Minimal-overhead launch for timed loops (no validation)."""
        self.L.macm_world_step(self.h, ctypes.c_void_p(actions_ptr), ctypes.byref(self._out),
                               ctypes.c_void_p(stream_handle))

    def rollout(self, actions: torch.Tensor):
        """K steps with actions given in advance ([K, E, N, 3] uint8/int8 or [K, E, N, 2] float32 on
        this device), one launch on the wave path (macm_world_rollout). Same results as K step()
        calls; the outputs hold the last step's values."""
        if actions.device != self.device or not actions.is_contiguous() or actions.dim() != 4:
            raise ValueError("actions must be a contiguous [K, E, N, A] tensor on the world's device")
        A = 3 if self.cfg.action_mode == _abi.ACTION_DISCRETE else 2
        ok = actions.dtype in (torch.uint8, torch.int8) if A == 3 else actions.dtype == torch.float32
        if not ok or tuple(actions.shape[1:]) != (self.E, self.N, A):
            raise ValueError(f"rollout actions must be [K,{self.E},{self.N},{A}] of the step's action dtype")
        _abi.check(self.L.macm_world_rollout(self.h, _ptr(actions), int(actions.shape[0]), ctypes.byref(self._out),
                                             self._stream()), "macm_world_rollout")
        return self.obs, self.nbr_id, self.reward, self.done

    def trajectory_buffers(self, n_steps: int) -> dict:
        """[n_steps, ...] output buffers for rollout_traj / rollout_bots_traj (reusable across calls)."""
        K, E, N = int(n_steps), self.E, self.N
        odt = torch.float64 if self.cfg.obs_f64 else torch.float32
        d = self.device
        return dict(obs=torch.empty((K, E, N, self.OD), dtype=odt, device=d),
                    nbr_id=torch.empty((K, E, N), dtype=torch.int32, device=d),
                    reward=torch.empty((K, E, N), dtype=torch.float32, device=d),
                    collided=torch.empty((K, E, N), dtype=torch.uint8, device=d),
                    done=torch.empty((K, E), dtype=torch.uint8, device=d))

    def _traj_out(self, traj: dict, K: int):
        return _abi.MacmOutputs(*[_ptr(t) for t in check_traj(traj, self._traj_spec(), K, self.device,
                                                              ("obs", "nbr_id", "reward", "collided", "done"))])

    def _traj_spec(self) -> dict:
        odt = torch.float64 if self.cfg.obs_f64 else torch.float32
        E, N = self.E, self.N
        return dict(obs=(odt, (E, N, self.OD)), nbr_id=(torch.int32, (E, N)), reward=(torch.float32, (E, N)),
                    collided=(torch.uint8, (E, N)), done=(torch.uint8, (E,)))

    def _keep_last(self, traj: dict, K: int) -> None:
        # the world's own buffers keep "the current step's outputs", as after step() / rollout()
        for k in ("obs", "nbr_id", "reward", "collided", "done"):
            if traj.get(k) is not None:
                getattr(self, k).copy_(traj[k][K - 1])

    def rollout_traj(self, actions: torch.Tensor, traj: dict = None) -> dict:
        """As rollout(), keeping every step's outputs (macm_world_rollout_traj): returns
        {obs [K,E,N,OD], nbr_id, reward, collided [K,E,N], done [K,E]} — the reference's (obs,
        rewards) of every env.step (mvmnt.py:140). ``traj``: buffers from trajectory_buffers(K)."""
        if actions.device != self.device or not actions.is_contiguous() or actions.dim() != 4:
            raise ValueError("actions must be a contiguous [K, E, N, A] tensor on the world's device")
        A = 3 if self.cfg.action_mode == _abi.ACTION_DISCRETE else 2
        ok = actions.dtype in (torch.uint8, torch.int8) if A == 3 else actions.dtype == torch.float32
        if not ok or tuple(actions.shape[1:]) != (self.E, self.N, A):
            raise ValueError(f"rollout actions must be [K,{self.E},{self.N},{A}] of the step's action dtype")
        K = int(actions.shape[0])
        traj = self.trajectory_buffers(K) if traj is None else traj
        out = self._traj_out(traj, K)
        _abi.check(self.L.macm_world_rollout_traj(self.h, _ptr(actions), K, ctypes.byref(out), self._stream()),
                   "macm_world_rollout_traj")
        if K > 0:
            self._keep_last(traj, K)
        return traj

    def rollout_bots_traj(self, actions: torch.Tensor, n_steps: int, traj: dict = None) -> dict:
        """As rollout_bots(), keeping every step's outputs and actions (macm_world_rollout_bots_traj):
        actions uint8 [n_steps + 1, E, N, 3], row 0 the first step's on entry; step k's bot actions
        land in row k + 1. Returns the trajectory dict of rollout_traj()."""
        K = int(n_steps)
        if (actions.device != self.device or not actions.is_contiguous() or actions.dtype != torch.uint8
                or tuple(actions.shape) != (K + 1, self.E, self.N, 3)):
            raise ValueError(f"actions must be a contiguous uint8 [{K + 1},{self.E},{self.N},3] tensor on the "
                             "world's device")
        traj = self.trajectory_buffers(K) if traj is None else traj
        out = self._traj_out(traj, K)
        _abi.check(self.L.macm_world_rollout_bots_traj(self.h, _ptr(actions), K, ctypes.byref(out), self._stream()),
                   "macm_world_rollout_bots_traj")
        if K > 0:
            self._keep_last(traj, K)
        return traj

    def traj_outputs(self, traj: dict):
        """The C-ABI outputs struct of trajectory buffers (trajectory_buffers(n_steps)), built once for
        repeated rollout_traj_raw calls (building it costs ~5 us of Python per call)."""
        return _abi.MacmOutputs(*[_ptr(traj.get(k)) for k in ("obs", "nbr_id", "reward", "collided", "done")])

    def rollout_traj_raw(self, actions_ptr: int, n_steps: int, traj, stream_handle: int) -> None:
        """Minimal-overhead trajectory rollout for timed loops (no validation); ``traj`` from
        trajectory_buffers(n_steps), or its traj_outputs(traj)."""
        out = traj if isinstance(traj, _abi.MacmOutputs) else self.traj_outputs(traj)
        self.L.macm_world_rollout_traj(self.h, ctypes.c_void_p(actions_ptr), int(n_steps), ctypes.byref(out),
                                       ctypes.c_void_p(stream_handle))

    def rollout_traj_launcher(self, actions_ptr: int, n_steps: int, traj, stream_handle: int):
        """rollout_traj_raw with every ctypes argument converted up front: a zero-argument callable
        that makes the launch (for timed loops; the buffers must outlive it)."""
        out = traj if isinstance(traj, _abi.MacmOutputs) else self.traj_outputs(traj)
        fn, ref = self.L.macm_world_rollout_traj, ctypes.byref(out)
        args = (self.h, ctypes.c_void_p(actions_ptr), ctypes.c_int(int(n_steps)), ref, ctypes.c_void_p(stream_handle))
        return lambda: fn(*args)

    def rollout_raw(self, actions_ptr: int, n_steps: int, stream_handle: int) -> None:
        """Minimal-overhead rollout for timed loops (no validation)."""
        self.L.macm_world_rollout(self.h, ctypes.c_void_p(actions_ptr), int(n_steps), ctypes.byref(self._out),
                                  ctypes.c_void_p(stream_handle))

    def rollout_bots(self, actions: torch.Tensor, n_steps: int):
        """n_steps of the closed loop step -> bots.flock -> step in one launch (macm_world_rollout_bots).
        actions: uint8 [E, N, 3] on this device, the first step's actions on entry (e.g.
        bots.flock_actions(self.obs)) and the bot's next actions on return."""
        if (actions.device != self.device or not actions.is_contiguous() or actions.dtype != torch.uint8
                or tuple(actions.shape) != (self.E, self.N, 3)):
            raise ValueError(f"actions must be a contiguous uint8 [{self.E},{self.N},3] tensor on the world's device")
        _abi.check(self.L.macm_world_rollout_bots(self.h, _ptr(actions), int(n_steps), ctypes.byref(self._out),
                                                  self._stream()), "macm_world_rollout_bots")
        return self.obs, self.nbr_id, self.reward, self.done

    def rollout_bots_raw(self, actions_ptr: int, n_steps: int, stream_handle: int) -> None:
        self.L.macm_world_rollout_bots(self.h, ctypes.c_void_p(actions_ptr), int(n_steps), ctypes.byref(self._out),
                                       ctypes.c_void_p(stream_handle))

    def observe(self):
        _abi.check(self.L.macm_world_observe(self.h, ctypes.byref(self._out_obs), self._stream()),
                   "macm_world_observe")
        return self.obs, self.nbr_id

    # -- state ---------------------------------------------------------------
    _STATE_KEYS = ("pos", "vel", "angle", "fat", "sleep", "targets", "contact_count", "contact_ab", "contact_imp",
                   "step_count", "time_passed")

    def state_buffers(self, stride=None):
        """Host arrays of get_state's layout; contact_ab / contact_imp rows of `stride` entries
        (default: max_contacts)."""
        E, N, T = self.E, self.N, self.T
        C = self.C if stride is None else int(stride)
        return dict(pos=np.zeros((E, N, 2), np.float32), vel=np.zeros((E, N, 2), np.float32),
                    angle=np.zeros((E, N), np.float32), fat=np.zeros((E, N, 4), np.float32),
                    sleep=np.zeros((E, N), np.float32), targets=np.zeros((E, T, 2), np.float32),
                    contact_count=np.zeros((E,), np.int32), contact_ab=np.zeros((E, C), np.uint32),
                    contact_imp=np.zeros((E, C, 2), np.float32), step_count=np.zeros((E,), np.int32),
                    time_passed=np.zeros((E,), np.float64))

    def _state_struct(self, arrs, stride):
        return _abi.MacmState(*[ctypes.c_void_p(arrs[k].ctypes.data) if arrs.get(k) is not None else None
                                for k in self._STATE_KEYS], int(stride))

    def get_state(self) -> dict:
        """The world's state as host arrays. The contact lists' rows hold max(contact_count)
        entries (at least 1), not max_contacts: only their used part crosses the bus (C can be
        large for N > 64); entries past an env's count are zero."""
        cnt = np.zeros((self.E,), np.int32)
        _abi.check(self.L.macm_world_get_state(self.h, ctypes.byref(self._state_struct({"contact_count": cnt}, 0)),
                                               self._stream()), "macm_world_get_state")
        stride = max(1, int(cnt.max(initial=0)))
        s = self.state_buffers(stride)
        _abi.check(self.L.macm_world_get_state(self.h, ctypes.byref(self._state_struct(s, stride)), self._stream()),
                   "macm_world_get_state")
        # entries past each env's contact_count are scratch: zero them so states compare/serialise cleanly
        idx = np.arange(stride)[None, :] >= s["contact_count"][:, None]
        s["contact_ab"][idx] = 0
        s["contact_imp"][idx] = 0
        return s

    def contact_list(self, e: int = 0) -> np.ndarray:
        """Env e's ordered contact list (uint32 a | b << 16, world-list order: the contacts that
        survive the next Collide, newest first), read without the rest of the state."""
        cnt = np.zeros((self.E,), np.int32)
        _abi.check(self.L.macm_world_get_state(self.h, ctypes.byref(self._state_struct({"contact_count": cnt}, 0)),
                                               self._stream()), "macm_world_get_state")
        stride = max(1, int(cnt.max(initial=0)))
        ab = np.zeros((self.E, stride), np.uint32)
        _abi.check(self.L.macm_world_get_state(self.h, ctypes.byref(self._state_struct(
            {"contact_count": cnt, "contact_ab": ab}, stride)), self._stream()), "macm_world_get_state")
        return ab[e, :int(cnt[e])].copy()

    def set_state(self, s: dict) -> None:
        """Inject a state (get_state's layout; the contact rows may have any length >= the counts,
        e.g. another world's max_contacts). A list longer than this world's capacity raises
        ValueError (truncating it would change the physics); the library validates the pairs on
        the device and takes nothing if any is invalid."""
        counts = np.asarray(s["contact_count"], dtype=np.int32)
        if counts.shape == (self.E,) and (counts.max(initial=0) > self.C or counts.min(initial=0) < 0):
            raise ValueError(f"contact_count must lie in [0, {self.C}] (this world's max_contacts); "
                             f"got [{int(counts.min())}, {int(counts.max())}]")
        ab = np.asarray(s["contact_ab"])
        stride = ab.shape[1] if ab.ndim == 2 else self.C
        ref = self.state_buffers(stride)
        arrs = {}
        for k, v in ref.items():
            a = np.ascontiguousarray(np.asarray(s[k], dtype=v.dtype))
            if a.shape != v.shape:
                raise ValueError(f"state[{k!r}] has shape {a.shape}, expected {v.shape}")
            arrs[k] = a
        _abi.check(self.L.macm_world_set_state(self.h, ctypes.byref(self._state_struct(arrs, stride)), self._stream()),
                   "macm_world_set_state")
        self.done.copy_(torch.from_numpy((arrs["time_passed"] > self.cfg.time_limit).astype(np.uint8)))

    def status(self) -> int:
        v = ctypes.c_int32()
        _abi.check(self.L.macm_world_status(self.h, ctypes.byref(v), self._stream()), "macm_world_status")
        return int(v.value)

    def counters(self) -> np.ndarray:
        out = (ctypes.c_int64 * 4)()
        _abi.check(self.L.macm_world_counters(self.h, out, self._stream()), "macm_world_counters")
        return np.array(list(out), np.int64)

    def launch_flags(self) -> int:
        """macm_world_info.launch_flags (MACM_LAUNCH_*): how the workgroup step launches, decided at the
        world's first step (the B -> C handoff)."""
        info = _abi.MacmWorldInfo()
        _abi.check(self.L.macm_world_info_get(self.h, ctypes.byref(info)), "macm_world_info_get")
        return int(info.launch_flags)

    def rollout_slices(self) -> int:
        """macm_world_info.rollout_slices: the env slices a workgroup-path rollout runs on streams of
        their own (0: none)."""
        info = _abi.MacmWorldInfo()
        _abi.check(self.L.macm_world_info_get(self.h, ctypes.byref(info)), "macm_world_info_get")
        return int(info.rollout_slices)

    def uses_handoff(self) -> bool:
        return bool(self.launch_flags() & _abi.LAUNCH_HANDOFF)

    def reward_sums(self):
        """(per-env reward totals [E] float64, their sum in env order) accumulated since creation or
        reset_counters, in the device's fixed order (macm_world_reward_sums; restated on the host by
        gym_macm.dist.pairwise_reward_sum). Synchronises the stream."""
        per_env = np.zeros((self.E,), np.float64)
        tot = ctypes.c_double()
        _abi.check(self.L.macm_world_reward_sums(self.h, ctypes.c_void_p(per_env.ctypes.data), ctypes.byref(tot),
                                                 self._stream()), "macm_world_reward_sums")
        return per_env, float(tot.value)

    def reset_counters(self) -> None:
        _abi.check(self.L.macm_world_reset_counters(self.h, self._stream()), "macm_world_reset_counters")

    def spilled(self) -> int:
        """Env-steps taken by the spill step (dense envs beyond the fast kernels' LDS capacities)."""
        v = ctypes.c_int64()
        _abi.check(self.L.macm_world_spilled(self.h, ctypes.byref(v), self._stream()), "macm_world_spilled")
        return int(v.value)

    def set_debug(self, flags: int) -> None:
        """Test hooks (macm_world_set_debug): _abi.DEBUG_FORCE_SPILL sends every env through the
        spill step; DEBUG_SWEEP_CELLS / DEBUG_SWEEP_ALL_PAIRS pick the workgroup path's pair sweep
        regardless of N (default: strip cells from N = 256); DEBUG_SPILL_POOL | slots << 8 shares
        that many working-set slots; DEBUG_SPILL_FAIL makes every slot request fail (the env is left
        unstepped with ST_SPILL_WAIT)."""
        _abi.check(self.L.macm_world_set_debug(self.h, int(flags)), "macm_world_set_debug")

    def check_status(self) -> None:
        """Raise MacmOverflowError if any env has a status bit set (synchronises the stream)."""
        st = self.status()
        if st:
            raise _abi.MacmOverflowError(_abi.E_OVERFLOW, "macm_world_status",
                                         f"status bits {st}: an env outgrew a capacity (max_contacts={self.C})")
