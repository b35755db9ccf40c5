"""Python handle over the TDM C-ABI (macm_tdm_*, include/macm.h).

Replaces the per-env ``TDM`` world of the reference (gym_macm/envs/combat.py:57-102,
one pybox2d ``b2World`` per env behind ``NoRender``) with one device-resident
world of E team-deathmatch envs; torch tensors are the device memory and torch's
current stream is the launch stream.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _abi
from .world import _ptr, check_traj


def tdm_config(n_agents=(1, 1), obs_f64=False, fresh_raycast=False, decay_mov_penalty=False, validate_actions=False,
               **overrides):
    """macm_tdm_config for TDM(n_agents=[...]) with combatSettings values
    (settings.py:149-177); keyword overrides use the config field names."""
    sizes = [int(n) for n in n_agents]
    if not 1 <= len(sizes) <= 4:
        raise ValueError("TDM supports 1 to 4 teams")
    c = _abi.tdm_config_from_defaults()
    c.n_teams = len(sizes)
    for t in range(4):
        c.team_size[t] = sizes[t] if t < len(sizes) else 0
    c.n_agents = sum(sizes)
    c.obs_f64 = 1 if obs_f64 else 0
    c.fresh_raycast = 1 if fresh_raycast else 0
    c.decay_mov_penalty = 1 if decay_mov_penalty else 0
    c.validate_actions = 1 if validate_actions else 0
    names = {f for f, _ in _abi.MacmTdmConfig._fields_}
    for k, v in overrides.items():
        if k not in names:
            raise TypeError(f"unknown TDM setting {k!r}")
        setattr(c, k, v)
    return c


class TdmWorld:
    """E independent TDM envs of one configuration on one GPU. Output tensors are
    owned by this object and overwritten by every call."""

    def __init__(self, cfg: _abi.MacmTdmConfig, n_envs: int = 1, device=None, host_outputs: bool = False):
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
        self.C = self.N * (self.N - 1) // 2
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            _abi.check(self.L.macm_tdm_create(ctypes.byref(cfg), self.E, device.index or 0, ctypes.byref(h)),
                       "macm_tdm_create")
        self.h = h
        odt = torch.float64 if cfg.obs_f64 else torch.float32
        E, N = self.E, self.N
        # host_outputs: pinned host outputs written by the kernels (zero-copy dict API)
        self.host_outputs = bool(host_outputs)
        kw = dict(pin_memory=True) if self.host_outputs else dict(device=device)
        self.obs = torch.empty((E, N, N - 1, 4), dtype=odt, **kw)
        self.mask = torch.empty((E, N, N - 1), dtype=torch.uint8, **kw)
        self.health = torch.empty((E, N), dtype=torch.float64, **kw)
        self.alive = torch.empty((E, N), dtype=torch.uint8, **kw)
        self.done = torch.zeros((E,), dtype=torch.uint8, **kw)
        self.winner = torch.full((E,), -1, dtype=torch.int32, **kw)
        if self.host_outputs:
            self.done.zero_()
        self._out = _abi.MacmTdmOutputs(_ptr(self.obs), _ptr(self.mask), _ptr(self.health), _ptr(self.alive),
                                        _ptr(self.done), _ptr(self.winner))
        team = []
        for t in range(cfg.n_teams):
            team += [t] * cfg.team_size[t]
        self.team = np.array(team, np.int32)

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.L.macm_tdm_destroy(h)
            except Exception:
                pass
            self.h = None

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def outputs(self):
        return self.obs, self.mask, self.health, self.alive, self.done, self.winner

    def reset(self, seed: int, env_offset: int = 0):
        """Env e := TDM(...) after random.seed(seed + env_offset + e); writes the initial obs."""
        _abi.check(self.L.macm_tdm_reset(self.h, int(seed), int(env_offset), ctypes.byref(self._out),
                                         self._stream()), "macm_tdm_reset")
        return self.outputs()

    def place(self, pos, angle):
        pos = np.ascontiguousarray(pos, np.float32).reshape(self.E, self.N, 2)
        angle = np.ascontiguousarray(angle, np.float32).reshape(self.E, self.N)
        _abi.check(self.L.macm_tdm_place(self.h, pos.ctypes.data, angle.ctypes.data, ctypes.byref(self._out),
                                         self._stream()), "macm_tdm_place")
        return self.outputs()

    def reset_envs(self, mask=None):
        """New episodes in the masked envs ([E] uint8/bool on this device, e.g.
        ``self.done``; None = all), continuing each env's random stream."""
        ptr = None
        if mask is not None:
            if mask.dtype == torch.bool:
                mask = mask.to(torch.uint8)
            if mask.device != self.device or tuple(mask.shape) != (self.E,) or mask.dtype != torch.uint8:
                raise ValueError(f"mask must be a uint8/bool tensor [{self.E}] on {self.device}")
            ptr = _ptr(mask.contiguous())
        _abi.check(self.L.macm_tdm_reset_envs(self.h, ptr, ctypes.byref(self._out), self._stream()),
                   "macm_tdm_reset_envs")
        return self.outputs()

    def step(self, actions: torch.Tensor):
        """actions: uint8 [E, N, 4] (forward, lateral, rotation, attack) on this device."""
        pinned_ok = self.host_outputs and actions.device.type == "cpu" and actions.is_pinned()
        if (actions.device != self.device and not pinned_ok) or not actions.is_contiguous():
            raise ValueError("actions must be a contiguous tensor on the world's device (or pinned host "
                             "memory with host_outputs)")
        if actions.dtype not in (torch.uint8, torch.int8) or tuple(actions.shape) != (self.E, self.N, 4):
            raise ValueError(f"TDM actions must be uint8 [{self.E},{self.N},4]")
        _abi.check(self.L.macm_tdm_step(self.h, _ptr(actions), ctypes.byref(self._out), self._stream()),
                   "macm_tdm_step")
        return self.outputs()

    def step_raw(self, actions_ptr: int, stream_handle: int) -> None:
        """Minimal-overhead launch for timed loops (no validation)."""
        self.L.macm_tdm_step(self.h, ctypes.c_void_p(actions_ptr), ctypes.byref(self._out),
                             ctypes.c_void_p(stream_handle))

    def rollout(self, actions: torch.Tensor):
        """K steps with actions given in advance (uint8 [K, E, N, 4] on this device) in one launch
        (macm_tdm_rollout); same results as K step() calls, the outputs hold the last step's."""
        if actions.device != self.device or not actions.is_contiguous() or actions.dim() != 4:
            raise ValueError("actions must be a contiguous [K, E, N, 4] tensor on the world's device")
        if actions.dtype not in (torch.uint8, torch.int8) or tuple(actions.shape[1:]) != (self.E, self.N, 4):
            raise ValueError(f"TDM rollout actions must be uint8 [K,{self.E},{self.N},4]")
        _abi.check(self.L.macm_tdm_rollout(self.h, _ptr(actions), int(actions.shape[0]), ctypes.byref(self._out),
                                           self._stream()), "macm_tdm_rollout")
        return self.outputs()

    _TRAJ_KEYS = ("obs", "mask", "health", "alive", "done", "winner")

    def trajectory_buffers(self, n_steps: int) -> dict:
        """[n_steps, ...] output buffers for rollout_traj / rollout_bots_traj (reusable across calls)."""
        K, E, N, d = int(n_steps), self.E, self.N, self.device
        odt = torch.float64 if self.cfg.obs_f64 else torch.float32
        return dict(obs=torch.empty((K, E, N, N - 1, 4), dtype=odt, device=d),
                    mask=torch.empty((K, E, N, N - 1), dtype=torch.uint8, device=d),
                    health=torch.empty((K, E, N), dtype=torch.float64, device=d),
                    alive=torch.empty((K, E, N), dtype=torch.uint8, device=d),
                    done=torch.empty((K, E), dtype=torch.uint8, device=d),
                    winner=torch.empty((K, E), dtype=torch.int32, device=d))

    def _traj_call(self, fn, name, actions, K, traj):
        traj = self.trajectory_buffers(K) if traj is None else traj
        odt = torch.float64 if self.cfg.obs_f64 else torch.float32
        E, N = self.E, self.N
        spec = dict(obs=(odt, (E, N, N - 1, 4)), mask=(torch.uint8, (E, N, N - 1)), health=(torch.float64, (E, N)),
                    alive=(torch.uint8, (E, N)), done=(torch.uint8, (E,)), winner=(torch.int32, (E,)))
        out = _abi.MacmTdmOutputs(*[_ptr(t) for t in check_traj(traj, spec, K, self.device, self._TRAJ_KEYS)])
        _abi.check(fn(self.h, _ptr(actions), K, ctypes.byref(out), self._stream()), name)
        if K > 0:  # the world's own buffers keep the current step's outputs
            for k in self._TRAJ_KEYS:
                if traj.get(k) is not None:
                    getattr(self, k).copy_(traj[k][K - 1])
        return traj

    def rollout_traj(self, actions: torch.Tensor, traj: dict = None) -> dict:
        """As rollout(), keeping every step's outputs (macm_tdm_rollout_traj): {obs [K,E,N,N-1,4],
        mask [K,E,N,N-1], health, alive [K,E,N], done, winner [K,E]}."""
        if actions.device != self.device or not actions.is_contiguous() or actions.dim() != 4:
            raise ValueError("actions must be a contiguous [K, E, N, 4] tensor on the world's device")
        if actions.dtype not in (torch.uint8, torch.int8) or tuple(actions.shape[1:]) != (self.E, self.N, 4):
            raise ValueError(f"TDM rollout actions must be uint8 [K,{self.E},{self.N},4]")
        return self._traj_call(self.L.macm_tdm_rollout_traj, "macm_tdm_rollout_traj", actions,
                               int(actions.shape[0]), traj)

    def rollout_bots_traj(self, actions: torch.Tensor, n_steps: int, traj: dict = None) -> dict:
        """As rollout_bots(), keeping every step's outputs and actions (macm_tdm_rollout_bots_traj):
        actions uint8 [n_steps + 1, E, N, 4], row 0 the first step's; step k's bot actions in row k + 1."""
        K = int(n_steps)
        if (actions.device != self.device or not actions.is_contiguous() or actions.dtype != torch.uint8
                or tuple(actions.shape) != (K + 1, self.E, self.N, 4)):
            raise ValueError(f"actions must be a contiguous uint8 [{K + 1},{self.E},{self.N},4] tensor on the "
                             "world's device")
        return self._traj_call(self.L.macm_tdm_rollout_bots_traj, "macm_tdm_rollout_bots_traj", actions, K, traj)

    def traj_outputs(self, traj: dict):
        """The C-ABI outputs struct of trajectory buffers, built once for repeated rollout_traj_raw calls."""
        return _abi.MacmTdmOutputs(*[_ptr(traj.get(k)) for k in self._TRAJ_KEYS])

    def rollout_traj_raw(self, actions_ptr: int, n_steps: int, traj, stream_handle: int) -> None:
        """Minimal-overhead trajectory rollout for timed loops (no validation); ``traj`` from
        trajectory_buffers(n_steps), or its traj_outputs(traj)."""
        out = traj if isinstance(traj, _abi.MacmTdmOutputs) else self.traj_outputs(traj)
        self.L.macm_tdm_rollout_traj(self.h, ctypes.c_void_p(actions_ptr), int(n_steps), ctypes.byref(out),
                                     ctypes.c_void_p(stream_handle))

    def rollout_traj_launcher(self, actions_ptr: int, n_steps: int, traj, stream_handle: int):
        """rollout_traj_raw with every ctypes argument converted up front: a zero-argument callable
        that makes the launch (for timed loops; the buffers must outlive it)."""
        out = traj if isinstance(traj, _abi.MacmTdmOutputs) else self.traj_outputs(traj)
        fn, ref = self.L.macm_tdm_rollout_traj, ctypes.byref(out)
        args = (self.h, ctypes.c_void_p(actions_ptr), ctypes.c_int(int(n_steps)), ref, ctypes.c_void_p(stream_handle))
        return lambda: fn(*args)

    def rollout_raw(self, actions_ptr: int, n_steps: int, stream_handle: int) -> None:
        """Minimal-overhead rollout for timed loops (no validation)."""
        self.L.macm_tdm_rollout(self.h, ctypes.c_void_p(actions_ptr), int(n_steps), ctypes.byref(self._out),
                                ctypes.c_void_p(stream_handle))

    def rollout_bots(self, actions: torch.Tensor, n_steps: int):
        """n_steps of the closed loop step -> bots.combat -> step in one launch (macm_tdm_rollout_bots);
        actions uint8 [E, N, 4]: the first step's on entry, the bot's next on return."""
        if (actions.device != self.device or not actions.is_contiguous() or actions.dtype != torch.uint8
                or tuple(actions.shape) != (self.E, self.N, 4)):
            raise ValueError(f"actions must be a contiguous uint8 [{self.E},{self.N},4] tensor on the world's device")
        _abi.check(self.L.macm_tdm_rollout_bots(self.h, _ptr(actions), int(n_steps), ctypes.byref(self._out),
                                                self._stream()), "macm_tdm_rollout_bots")
        return self.outputs()

    def rollout_bots_raw(self, actions_ptr: int, n_steps: int, stream_handle: int) -> None:
        self.L.macm_tdm_rollout_bots(self.h, ctypes.c_void_p(actions_ptr), int(n_steps), ctypes.byref(self._out),
                                     ctypes.c_void_p(stream_handle))

    def observe(self):
        _abi.check(self.L.macm_tdm_observe(self.h, ctypes.byref(self._out), self._stream()), "macm_tdm_observe")
        return self.outputs()

    def state_buffers(self, stride=None):
        """Host arrays of get_state's layout; contact_ab / contact_imp rows of `stride` entries
        (default: C = every pair)."""
        E, N = self.E, self.N
        C = self.C if stride is None else int(stride)
        return dict(pos=np.zeros((E, N, 2), np.float32), vel=np.zeros((E, N, 2), np.float32),
                    angle=np.zeros((E, N), np.float32), fat=np.zeros((E, N, 4), np.float32),
                    sleep=np.zeros((E, N), np.float32), health=np.zeros((E, N), np.float64),
                    cd_atk=np.zeros((E, N), np.float64), cd_mov=np.zeros((E, N), np.float64),
                    alive=np.zeros((E, N), np.uint8), listener=np.zeros((E, 2), np.int32),
                    contact_count=np.zeros((E,), np.int32), contact_ab=np.zeros((E, C), np.uint32),
                    contact_imp=np.zeros((E, C, 2), np.float32), step_count=np.zeros((E,), np.int32),
                    time_passed=np.zeros((E,), np.float64), done=np.zeros((E,), np.uint8),
                    winner=np.zeros((E,), np.int32))

    @staticmethod
    def _state_struct(arrs, stride):
        return _abi.MacmTdmState(*[ctypes.c_void_p(arrs[k].ctypes.data) if arrs.get(k) is not None else None
                                   for k in _abi.TDM_STATE_FIELDS], int(stride))

    def get_state(self) -> dict:
        """The world's state as host arrays. The contact lists' rows hold max(contact_count) entries
        (at least 1), not C = N(N-1)/2: only their used part crosses the bus (C is
        523,776 at N = 1024); entries past an env's count are zero."""
        cnt = np.zeros((self.E,), np.int32)
        _abi.check(self.L.macm_tdm_get_state(self.h, ctypes.byref(self._state_struct({"contact_count": cnt}, 0)),
                                             self._stream()), "macm_tdm_get_state")
        stride = max(1, int(cnt.max(initial=0)))
        s = self.state_buffers(stride)
        _abi.check(self.L.macm_tdm_get_state(self.h, ctypes.byref(self._state_struct(s, stride)), self._stream()),
                   "macm_tdm_get_state")
        idx = np.arange(stride)[None, :] >= s["contact_count"][:, None]
        s["contact_ab"][idx] = 0
        s["contact_imp"][idx] = 0
        return s

    def set_state(self, s: dict) -> None:
        """Inject a state (get_state's layout; the contact rows may have any length >= the counts);
        the library validates the pairs on the device and takes nothing if any is invalid."""
        counts = np.asarray(s["contact_count"], dtype=np.int32)
        if counts.shape == (self.E,) and (counts.max(initial=0) > self.C or counts.min(initial=0) < 0):
            raise ValueError(f"contact_count must lie in [0, {self.C}]")
        ab = np.asarray(s["contact_ab"])
        stride = ab.shape[1] if ab.ndim == 2 else self.C
        ref = self.state_buffers(stride)
        arrs = {}
        for k, v in ref.items():
            a = np.ascontiguousarray(np.asarray(s[k], dtype=v.dtype))
            if a.shape != v.shape:
                raise ValueError(f"state[{k!r}] has shape {a.shape}, expected {v.shape}")
            arrs[k] = a
        _abi.check(self.L.macm_tdm_set_state(self.h, ctypes.byref(self._state_struct(arrs, stride)), self._stream()),
                   "macm_tdm_set_state")

    def status(self) -> int:
        v = ctypes.c_int32()
        _abi.check(self.L.macm_tdm_status(self.h, ctypes.byref(v), self._stream()), "macm_tdm_status")
        return int(v.value)

    def check_status(self) -> None:
        """Raise MacmOverflowError if any env has a status bit set (synchronises the stream). Dense
        envs take the spill step (no capacity bit); only a pooled working set's SPILL_WAIT remains."""
        st = self.status()
        if st:
            raise _abi.MacmOverflowError(_abi.E_OVERFLOW, "macm_tdm_status",
                                         f"status bits {st}: an env was not stepped as the reference")

    def spilled(self) -> int:
        """Env-steps taken by the spill step (envs beyond 256 touching contacts or 16 per body)."""
        v = ctypes.c_int64()
        _abi.check(self.L.macm_tdm_spilled(self.h, ctypes.byref(v), self._stream()), "macm_tdm_spilled")
        return int(v.value)

    def launch_flags(self) -> int:
        """MACM_LAUNCH_* of the next step / rollout (macm_tdm_launch_flags): LAUNCH_SPLIT_OBS when the
        observation is written by its own kernel from pose snapshots (fewer than 1024 envs),
        LAUNCH_TAIL_OBS when trajectory rollouts take the tail observation (fewer than 2048 envs)."""
        f = self.L.macm_tdm_launch_flags(self.h)
        _abi.check(min(f, 0), "macm_tdm_launch_flags")
        return int(f)

    def reserve(self, n_steps: int) -> None:
        """Allocate ahead what trajectory rollouts of up to n_steps steps need (macm_tdm_reserve: the tail
        observation's snapshots), so that the rollout itself does not reallocate."""
        _abi.check(self.L.macm_tdm_reserve(self.h, int(n_steps), self._stream()), "macm_tdm_reserve")

    def set_debug(self, flags: int) -> None:
        """Test hooks (macm_tdm_set_debug): _abi.DEBUG_FORCE_SPILL sends every env through the spill
        step; DEBUG_SPILL_POOL | slots << 8 shares that many working-set slots; DEBUG_SPILL_FAIL makes
        every slot request fail (the env is left unstepped with ST_SPILL_WAIT)."""
        _abi.check(self.L.macm_tdm_set_debug(self.h, int(flags)), "macm_tdm_set_debug")

    def counters(self) -> np.ndarray:
        out = (ctypes.c_int64 * 4)()
        _abi.check(self.L.macm_tdm_counters(self.h, out, self._stream()), "macm_tdm_counters")
        return np.array(list(out), np.int64)
