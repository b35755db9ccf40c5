"""ctypes wrapper of the CPU oracle (liboracle_flock.so).

ORACLE / TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, as the checker or the timed CPU baseline —
never by the product package (gym-macm_amd/).

Two layers:
  * ``OracleFlock`` — E independent reference envs (gym_macm/envs/mvmnt.py restated
    in C over b2lite), same config struct and state layout as the HIP world.
  * ``B2World`` — the low-level b2lite world (Box2D 2.3 subset) used by
    tests/golden/box2d_facade.py to run the reference's own Python env code.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from ctypes import POINTER, c_double, c_float, c_int, c_int32, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
# MACM_ORACLE_LIB: an alternative build of the same sources, e.g. the sanitizer leg
# (make -C oracle asan -> oracle/_asan/liboracle_flock.so, tools/asan_oracle.sh)
LIB = os.environ.get("MACM_ORACLE_LIB") or os.path.join(HERE, "liboracle_flock.so")

def _load_abi():
    # ctypes mirror of include/macm.h, loaded by path so that this module never
    # shadows (or is shadowed by) a `gym_macm` package: the golden generator
    # imports the reference's gym_macm in the same process.
    import importlib.util
    path = os.path.join(REPO, "gym-macm_amd", "gym_macm", "_abi.py")
    spec = importlib.util.spec_from_file_location("_macm_abi_mirror", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["_macm_abi_mirror"] = mod
    spec.loader.exec_module(mod)
    return mod


_abi = _load_abi()

_L = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB):
        build()
    L = ctypes.CDLL(LIB)
    P = POINTER
    sig = {
        "fo_create": (c_void_p, [c_void_p, P(c_int32), c_int, c_uint64, c_int64]),
        "fo_free": (None, [c_void_p]),
        "fo_obs_dim": (c_int, [c_void_p]),
        "fo_observe": (None, [c_void_p, P(c_double), P(c_int32)]),
        "fo_step": (None, [c_void_p, c_void_p, P(c_double), P(c_int32), P(c_double), P(c_uint8),
                           P(c_uint8), c_int]),
        "fo_contacts": (c_int, [c_void_p, c_int, P(c_int), c_int]),
        "fo_get_state": (None, [c_void_p] + [P(c_float)] * 6 + [P(c_int32), P(c_uint32), P(c_float),
                                                                 c_int, P(c_int32), P(c_double)]),
        "fo_set_state": (None, [c_void_p] + [P(c_float)] * 6 + [P(c_int32), P(c_uint32), P(c_float),
                                                                 c_int, P(c_int32), P(c_double)]),
        "fo_world_new": (c_void_p, []),
        "b2l_world_free": (None, [c_void_p]),
        "b2l_world_set_flags": (None, [c_void_p, c_int, c_int, c_int]),
        "b2l_create_body": (c_int, [c_void_p, c_void_p]),
        "b2l_body_get": (None, [c_void_p, c_int, P(c_float)]),
        "b2l_body_get_fat": (None, [c_void_p, c_int, P(c_float)]),
        "b2l_body_set_transform": (None, [c_void_p, c_int, c_float, c_float, c_float]),
        "b2l_body_apply_force": (None, [c_void_p, c_int, c_float, c_float, c_float, c_float, c_int]),
        "b2l_world_step": (None, [c_void_p, c_float, c_int, c_int]),
        "b2l_world_clear_forces": (None, [c_void_p]),
        "b2l_world_contacts": (c_int, [c_void_p, P(c_int), c_int]),
        "b2l_world_contact_impulses": (c_int, [c_void_p, P(c_float), c_int]),
        "b2l_body_set_active": (None, [c_void_p, c_int, c_int]),
        "b2l_body_active": (c_int, [c_void_p, c_int]),
        "b2l_world_raycast": (c_int, [c_void_p, c_float, c_float, c_float, c_float, P(c_float)]),
        "to_create": (c_void_p, [c_void_p, c_int, c_uint64, c_int64]),
        "to_free": (None, [c_void_p]),
        "to_n_agents": (c_int, [c_void_p]),
        "to_observe": (None, [c_void_p, P(c_double), P(c_uint8)]),
        "to_step": (None, [c_void_p, c_void_p, P(c_double), P(c_uint8), P(c_double), P(c_uint8), P(c_uint8),
                           P(c_int32), c_int]),
        "to_get_extras": (None, [c_void_p, P(c_double), P(c_double), P(c_int32)]),
        "to_world": (c_void_p, [c_void_p, c_int]),
        "to_reset_envs": (None, [c_void_p, c_void_p]),
        "fo_reset_envs": (None, [c_void_p, c_void_p]),
        "to_get_state": (None, [c_void_p] + [c_void_p] * 13 + [c_int] + [c_void_p] * 4),
        "gs_levels": (None, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float, c_void_p]),
        "to_set_state": (None, [c_void_p] + [c_void_p] * 13 + [c_int] + [c_void_p] * 4),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _L = L
    return L


def _p(a, ct):
    return a.ctypes.data_as(POINTER(ct)) if a is not None else None


class BodyDef(ctypes.Structure):
    _fields_ = [("x", c_float), ("y", c_float), ("angle", c_float), ("linear_damping", c_float),
                ("fixed_rotation", c_int), ("allow_sleep", c_int), ("radius", c_float),
                ("density", c_float), ("friction", c_float), ("restitution", c_float)]


class OracleFlock:
    """E reference Flock envs on the CPU; env e == Flock after random.seed(seed + env_offset + e)."""

    def __init__(self, cfg: _abi.MacmConfig, targets_idx, n_envs: int, seed: int, env_offset: int = 0):
        self.L = lib()
        self.cfg = cfg
        self.E, self.N, self.T = n_envs, cfg.n_agents, cfg.n_targets
        ti = np.zeros(self.N, np.int32) if targets_idx is None else np.ascontiguousarray(targets_idx, np.int32)
        # cfg may come from either copy of the ABI mirror: pass its address
        self.h = self.L.fo_create(ctypes.addressof(cfg), _p(ti, c_int32), n_envs, seed, env_offset)
        if not self.h:
            raise ValueError("fo_create rejected the config")
        self.OD = self.L.fo_obs_dim(self.h)

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.L.fo_free(h)
            self.h = None

    def reset_envs(self, mask=None):
        """This build's working Flock.reset for the masked envs (next poses from each
        env's stream, targets kept, fresh world)."""
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        self.L.fo_reset_envs(self.h, None if m is None else m.ctypes.data)

    def observe(self):
        obs = np.zeros((self.E, self.N, self.OD), np.float64)
        nbr = np.zeros((self.E, self.N), np.int32)
        self.L.fo_observe(self.h, _p(obs, c_double), _p(nbr, c_int32))
        return obs, nbr

    def step(self, actions: np.ndarray, n_threads: int = 1):
        if self.cfg.action_mode == _abi.ACTION_DISCRETE:
            a = np.ascontiguousarray(actions, np.uint8).reshape(self.E, self.N, 3)
        else:
            a = np.ascontiguousarray(actions, np.float32).reshape(self.E, self.N, 2)
        obs = np.zeros((self.E, self.N, self.OD), np.float64)
        nbr = np.zeros((self.E, self.N), np.int32)
        rew = np.zeros((self.E, self.N), np.float64)
        col = np.zeros((self.E, self.N), np.uint8)
        done = np.zeros((self.E,), np.uint8)
        self.L.fo_step(self.h, a.ctypes.data, _p(obs, c_double), _p(nbr, c_int32), _p(rew, c_double),
                       _p(col, c_uint8), _p(done, c_uint8), n_threads)
        return dict(obs=obs, nbr_id=nbr, reward=rew, collided=col, done=done)

    def step_raw(self, actions: np.ndarray, bufs: dict, n_threads: int) -> None:
        """Allocation-free step for the timed CPU baseline."""
        self.L.fo_step(self.h, actions.ctypes.data, _p(bufs["obs"], c_double), _p(bufs["nbr_id"], c_int32),
                       _p(bufs["reward"], c_double), None, None, n_threads)

    def contacts(self, e: int) -> np.ndarray:
        n = self.L.fo_contacts(self.h, e, None, 0)
        out = np.zeros((max(n, 1), 3), np.int32)
        self.L.fo_contacts(self.h, e, out.ctypes.data_as(POINTER(c_int)), n)
        return out[:n]

    def get_state(self, max_contacts: int) -> dict:
        E, N, T, C = self.E, self.N, self.T, max_contacts
        s = dict(pos=np.zeros((E, N, 2), np.float32), vel=np.zeros((E, N, 2), np.float32),
                 angle=np.zeros((E, N), np.float32), fat=np.zeros((E, N, 4), np.float32),
                 sleep=np.zeros((E, N), np.float32), targets=np.zeros((E, T, 2), np.float32),
                 contact_count=np.zeros((E,), np.int32), contact_ab=np.zeros((E, C), np.uint32),
                 contact_imp=np.zeros((E, C, 2), np.float32), step_count=np.zeros((E,), np.int32),
                 time_passed=np.zeros((E,), np.float64))
        self.L.fo_get_state(self.h, *[_p(s[k], c_float) for k in ("pos", "vel", "angle", "fat", "sleep", "targets")],
                            _p(s["contact_count"], c_int32), _p(s["contact_ab"], c_uint32),
                            _p(s["contact_imp"], c_float), C, _p(s["step_count"], c_int32),
                            _p(s["time_passed"], c_double))
        if int(s["contact_count"].max(initial=0)) > C:
            raise OverflowError("oracle contact list exceeds max_contacts")
        return s

    def levels(self) -> np.ndarray:
        """[E, 4] int32 of the state the next step starts from (oracle/gs_levels.c): touching contacts,
        Gauss-Seidel levels per pass in Box2D's island order (the deepest island), islands, contacts of
        the largest island. A measurement for the chain floor, not part of the restatement."""
        cap = max(1, max(self.L.fo_contacts(self.h, e, None, 0) for e in range(self.E)))
        st = self.get_state(cap)
        out = np.zeros((self.E, 4), np.int32)
        rr = np.float32(2 * self.cfg.radius) ** 2
        self.L.gs_levels(self.E, self.N, cap, st["pos"].ctypes.data, st["contact_count"].ctypes.data,
                         st["contact_ab"].ctypes.data, float(rr), out.ctypes.data)
        return out

    def set_state(self, s: dict) -> None:
        C = s["contact_ab"].shape[1]
        arr = {k: np.ascontiguousarray(v) for k, v in s.items()}
        self.L.fo_set_state(self.h, *[_p(arr[k], c_float) for k in ("pos", "vel", "angle", "fat", "sleep", "targets")],
                            _p(arr["contact_count"], c_int32), _p(arr["contact_ab"], c_uint32),
                            _p(arr["contact_imp"], c_float), C, _p(arr["step_count"], c_int32),
                            _p(arr["time_passed"], c_double))


class B2World:
    """Low-level b2lite world (one Box2D world) for the golden-vector facade."""

    def __init__(self):
        self.L = lib()
        self.h = self.L.fo_world_new()
        self._buf = (c_float * 7)()

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.L.b2l_world_free(h)
            self.h = None

    def create_body(self, x, y, angle, radius, density, friction, linear_damping, fixed_rotation):
        d = BodyDef(x, y, angle, linear_damping, int(fixed_rotation), 1, radius, density, friction, 0.0)
        return self.L.b2l_create_body(self.h, ctypes.byref(d))

    def body(self, i):
        self.L.b2l_body_get(self.h, i, self._buf)
        return tuple(self._buf)

    def set_transform(self, i, x, y, a):
        self.L.b2l_body_set_transform(self.h, i, x, y, a)

    def apply_force(self, i, fx, fy, px, py, wake):
        self.L.b2l_body_apply_force(self.h, i, fx, fy, px, py, int(wake))

    def step(self, dt, vi, pi, warm=True, cont=True, sub=False):
        self.L.b2l_world_set_flags(self.h, int(warm), int(cont), int(sub))
        self.L.b2l_world_step(self.h, dt, vi, pi)

    def clear_forces(self):
        self.L.b2l_world_clear_forces(self.h)

    def set_active(self, i, flag):
        self.L.b2l_body_set_active(self.h, i, int(flag))

    def active(self, i):
        return self.L.b2l_body_active(self.h, i)

    def raycast(self, x1, y1, x2, y2):
        fr = c_float()
        hit = self.L.b2l_world_raycast(self.h, x1, y1, x2, y2, ctypes.byref(fr))
        return hit, fr.value

    def contacts(self):
        n = self.L.b2l_world_contacts(self.h, None, 0)
        out = (c_int * (3 * max(n, 1)))()
        self.L.b2l_world_contacts(self.h, out, n)
        return [(out[3 * k], out[3 * k + 1], out[3 * k + 2]) for k in range(n)]


class OracleTDM:
    """E reference TDM envs on the CPU (oracle/tdm_oracle.c); env e == TDM after
    random.seed(seed + env_offset + e), with combat.py's missing names patched in."""

    def __init__(self, cfg, n_envs: int, seed: int, env_offset: int = 0):
        self.L = lib()
        self.cfg = cfg
        self.h = self.L.to_create(ctypes.addressof(cfg), n_envs, seed, env_offset)
        if not self.h:
            raise ValueError("to_create rejected the config")
        self.E = n_envs
        self.N = self.L.to_n_agents(self.h)

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            self.L.to_free(h)
            self.h = None

    def _bufs(self):
        E, N = self.E, self.N
        return (np.zeros((E, N, N - 1, 4), np.float64), np.zeros((E, N, N - 1), np.uint8))

    def observe(self):
        obs, mask = self._bufs()
        self.L.to_observe(self.h, _p(obs, c_double), _p(mask, c_uint8))
        return obs, mask

    def step(self, actions, n_threads=1):
        E, N = self.E, self.N
        a = np.ascontiguousarray(actions, np.uint8).reshape(E, N, 4)
        obs, mask = self._bufs()
        health = np.zeros((E, N), np.float64)
        alive = np.zeros((E, N), np.uint8)
        done = np.zeros((E,), np.uint8)
        winner = np.zeros((E,), np.int32)
        self.L.to_step(self.h, a.ctypes.data, _p(obs, c_double), _p(mask, c_uint8), _p(health, c_double),
                       _p(alive, c_uint8), _p(done, c_uint8), _p(winner, c_int32), n_threads)
        return dict(obs=obs, mask=mask, health=health, alive=alive, done=done, winner=winner)

    def reset_envs(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        self.L.to_reset_envs(self.h, None if m is None else m.ctypes.data)

    def extras(self):
        E, N = self.E, self.N
        cd_atk = np.zeros((E, N), np.float64)
        cd_mov = np.zeros((E, N), np.float64)
        lis = np.zeros((E, 2), np.int32)
        self.L.to_get_extras(self.h, _p(cd_atk, c_double), _p(cd_mov, c_double), _p(lis, c_int32))
        return dict(cd_atk=cd_atk, cd_mov=cd_mov, listener=lis)

    def state_buffers(self):
        E, N = self.E, self.N
        C = N * (N - 1) // 2
        return dict(pos=np.zeros((E, N, 2), np.float32), vel=np.zeros((E, N, 2), np.float32),
                    angle=np.zeros((E, N), np.float32), fat=np.zeros((E, N, 4), np.float32),
                    sleep=np.zeros((E, N), np.float32), health=np.zeros((E, N), np.float64),
                    cd_atk=np.zeros((E, N), np.float64), cd_mov=np.zeros((E, N), np.float64),
                    alive=np.zeros((E, N), np.uint8), listener=np.zeros((E, 2), np.int32),
                    contact_count=np.zeros((E,), np.int32), contact_ab=np.zeros((E, C), np.uint32),
                    contact_imp=np.zeros((E, C, 2), np.float32), step_count=np.zeros((E,), np.int32),
                    time_passed=np.zeros((E,), np.float64), done=np.zeros((E,), np.uint8),
                    winner=np.zeros((E,), np.int32))

    _ORDER = ("pos", "vel", "angle", "fat", "sleep", "health", "cd_atk", "cd_mov", "alive", "listener",
              "contact_count", "contact_ab", "contact_imp")
    _TAIL = ("step_count", "time_passed", "done", "winner")

    def get_state(self):
        """State in the macm_tdm_state layout (contact list capacity N(N-1)/2)."""
        st = self.state_buffers()
        C = self.N * (self.N - 1) // 2
        self.L.to_get_state(self.h, *[st[k].ctypes.data for k in self._ORDER], C,
                            *[st[k].ctypes.data for k in self._TAIL])
        return st

    def set_state(self, st):
        C = self.N * (self.N - 1) // 2
        ref = self.state_buffers()
        arrs = {k: np.ascontiguousarray(st[k], ref[k].dtype).reshape(ref[k].shape) for k in ref}
        self.L.to_set_state(self.h, *[arrs[k].ctypes.data for k in self._ORDER], C,
                            *[arrs[k].ctypes.data for k in self._TAIL])

    def bodies(self, e):
        """[(x, y, angle, vx, vy, sleep, awake)] of env e."""
        w = self.L.to_world(self.h, e)
        buf = (c_float * 7)()
        out = []
        for i in range(self.N):
            self.L.b2l_body_get(w, i, buf)
            out.append(tuple(buf))
        return np.array(out, np.float32)
