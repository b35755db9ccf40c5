"""ctypes mirror of include/macm.h and the loader for libmacm_hip.so.

The product path is the HIP library. There is no CPU fallback: if the library is
missing or fails to load, :func:`lib` raises ``MacmLibraryError`` with the reason.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_double, c_float, c_int, c_int32, c_int64,
                    c_uint8, c_uint64, c_void_p)

ACTION_DISCRETE, ACTION_CONTINUOUS = 0, 1
REWARD_BINARY, REWARD_LINEAR = 0, 1
COORD_POLAR, COORD_CARTESIAN = 0, 1

ST_CONTACT_OVERFLOW, ST_TOUCH_OVERFLOW, ST_DEGREE_OVERFLOW, ST_INVALID_ACTION, ST_SPILL_WAIT = 1, 2, 4, 8, 16
ST_HANDOFF = 32
DEBUG_FORCE_SPILL = 1
DEBUG_SWEEP_CELLS = 2
DEBUG_SWEEP_ALL_PAIRS = 4
DEBUG_SPILL_POOL = 8  # | slots << 8
DEBUG_SPILL_FAIL = 16  # no spill slot is ever free (SPILL_WAIT test hook)
E_INVALID, E_OVERFLOW = -1, -5

_ERRORS = {
    -1: "MACM_E_INVALID",
    -2: "MACM_E_OOM",
    -3: "MACM_E_HIP",
    -4: "MACM_E_UNSUPPORTED",
    -5: "MACM_E_OVERFLOW",
}


class MacmConfig(Structure):
    _fields_ = [
        ("n_agents", c_int32),
        ("n_targets", c_int32),
        ("action_mode", c_int32),
        ("reward_mode", c_int32),
        ("coord", c_int32),
        ("velocity_iterations", c_int32),
        ("position_iterations", c_int32),
        ("warm_starting", c_int32),
        ("obs_f64", c_int32),
        ("validate_actions", c_int32),
        ("hz", c_double),
        ("start_spread", c_double),
        ("start_point", c_double * 2),
        ("agent_rotation_speed", c_double),
        ("agent_force", c_double),
        ("time_limit", c_double),
        ("reward_radius", c_double),
        ("target_mindist", c_double),
        ("target_maxdist", c_double),
        ("radius", c_float),
        ("density", c_float),
        ("friction", c_float),
        ("linear_damping", c_float),
    ]


class MacmOutputs(Structure):
    _fields_ = [
        ("obs", c_void_p),
        ("nbr_id", c_void_p),
        ("reward", c_void_p),
        ("collided", c_void_p),
        ("done", c_void_p),
    ]


class MacmState(Structure):
    _fields_ = [(n, c_void_p) for n in (
        "pos", "vel", "angle", "fat", "sleep", "targets", "contact_count", "contact_ab",
        "contact_imp", "step_count", "time_passed")] + [("contact_stride", c_int64)]


LAUNCH_HANDOFF = 1  # macm_world_info.launch_flags
LAUNCH_SPLIT_OBS = 2  # macm_tdm_launch_flags
LAUNCH_TAIL_OBS = 4  # macm_tdm_launch_flags: trajectory rollouts take the tail observation


class MacmWorldInfo(Structure):
    _fields_ = [
        ("n_envs", c_int32),
        ("n_agents", c_int32),
        ("n_targets", c_int32),
        ("obs_dim", c_int32),
        ("max_contacts", c_int32),
        ("max_touching", c_int32),
        ("device", c_int32),
        ("spill_slots", c_int32),
        ("launch_flags", c_int32),
        ("rollout_slices", c_int32),
    ]


class MacmTdmConfig(Structure):
    _fields_ = [
        ("n_teams", c_int32),
        ("team_size", c_int32 * 4),
        ("n_agents", c_int32),
        ("velocity_iterations", c_int32),
        ("position_iterations", c_int32),
        ("warm_starting", c_int32),
        ("obs_f64", c_int32),
        ("fresh_raycast", c_int32),
        ("decay_mov_penalty", c_int32),
        ("validate_actions", c_int32),
        ("_pad", c_int32),
        ("hz", c_double),
        ("world_width", c_double),
        ("world_height", c_double),
        ("agent_rotation_speed", c_double),
        ("agent_force", c_double),
        ("percent_mov_penalty", c_double),
        ("melee_range", c_double),
        ("melee_dmg", c_double),
        ("init_health", c_double),
        ("cooldown_atk", c_double),
        ("cooldown_mov_penalty", c_double),
        ("time_limit", c_double),
        ("radius", c_float),
        ("density", c_float),
        ("friction", c_float),
        ("linear_damping", c_float),
    ]


class MacmTdmOutputs(Structure):
    _fields_ = [(n, c_void_p) for n in ("obs", "mask", "health", "alive", "done", "winner")]


TDM_STATE_FIELDS = ("pos", "vel", "angle", "fat", "sleep", "health", "cd_atk", "cd_mov", "alive", "listener",
                    "contact_count", "contact_ab", "contact_imp", "step_count", "time_passed", "done", "winner")


class MacmTdmState(Structure):
    _fields_ = [(n, c_void_p) for n in TDM_STATE_FIELDS] + [("contact_stride", ctypes.c_int64)]


def tdm_config_from_defaults() -> "MacmTdmConfig":
    """macm_tdm_config_default without the HIP library (used by the CPU oracle too)."""
    import math
    c = MacmTdmConfig()
    c.n_teams = 2
    c.team_size[0] = 1
    c.team_size[1] = 1
    c.n_agents = 2
    c.velocity_iterations, c.position_iterations, c.warm_starting = 8, 3, 1
    c.hz, c.world_width, c.world_height = 60.0, 30.0, 30.0
    c.agent_rotation_speed = 0.8 * (2 * math.pi)
    c.agent_force, c.percent_mov_penalty = 20.0, 0.2
    c.melee_range, c.melee_dmg, c.init_health = 2.0, 0.25, 1.0
    c.cooldown_atk, c.cooldown_mov_penalty, c.time_limit = 1.0, 0.5, 60.0
    c.radius, c.density, c.friction, c.linear_damping = 0.5, 1.0, 0.3, 5.0
    return c


class MacmLibraryError(RuntimeError):
    """The HIP library failed: it could not be loaded (the product path refuses to run without
    it), or one of its calls returned an error (MacmError)."""


class MacmError(MacmLibraryError):
    """A C-ABI call returned a negative MACM_E_* status; ``code`` holds it."""

    def __init__(self, code: int, fn: str, msg: str):
        super().__init__(f"{fn} failed: {_ERRORS.get(code, code)}: {msg}")
        self.code = code


class MacmOverflowError(MacmError):
    """MACM_E_OVERFLOW: an env outgrew a capacity in an earlier step, so the results since then
    are not the reference's (the step refuses to continue until reset / place / set_state).
    Detection is eventual: steps queued behind the overflowing one still run, and the first call
    that sees the device's host-mapped status word raises; check_status() synchronises and is exact."""


class MacmInvalidActionError(MacmError):
    """MACM_E_INVALID from a step with validate_actions: an action outside the action space
    (the reference's ``assert self.action_space.contains(actions)``); no env was stepped."""


PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # gym-macm_amd/
LIB_PATH = os.environ.get("MACM_LIB", os.path.join(PKG_ROOT, "libmacm_hip.so"))

# Exported symbols and their signatures (must equal include/macm.h).
SIGNATURES = {
    "macm_version": (c_char_p, []),
    "macm_abi_version": (c_int, []),
    "macm_last_error": (c_char_p, []),
    "macm_config_default": (c_int, [POINTER(MacmConfig)]),
    "macm_world_create": (c_int, [POINTER(MacmConfig), POINTER(c_int32), c_int32, c_int32, c_int32,
                                  POINTER(c_void_p)]),
    "macm_world_destroy": (c_int, [c_void_p]),
    "macm_world_info_get": (c_int, [c_void_p, POINTER(MacmWorldInfo)]),
    "macm_world_reset": (c_int, [c_void_p, c_uint64, c_int64, POINTER(MacmOutputs), c_void_p]),
    "macm_world_place": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, POINTER(MacmOutputs), c_void_p]),
    "macm_world_reset_envs": (c_int, [c_void_p, c_void_p, POINTER(MacmOutputs), c_void_p]),
    "macm_world_step": (c_int, [c_void_p, c_void_p, POINTER(MacmOutputs), c_void_p]),
    "macm_world_rollout": (c_int, [c_void_p, c_void_p, c_int, POINTER(MacmOutputs), c_void_p]),
    "macm_world_rollout_bots": (c_int, [c_void_p, c_void_p, c_int, POINTER(MacmOutputs), c_void_p]),
    "macm_world_rollout_traj": (c_int, [c_void_p, c_void_p, c_int, POINTER(MacmOutputs), c_void_p]),
    "macm_world_rollout_bots_traj": (c_int, [c_void_p, c_void_p, c_int, POINTER(MacmOutputs), c_void_p]),
    "macm_world_observe": (c_int, [c_void_p, POINTER(MacmOutputs), c_void_p]),
    "macm_world_get_state": (c_int, [c_void_p, POINTER(MacmState), c_void_p]),
    "macm_world_set_state": (c_int, [c_void_p, POINTER(MacmState), c_void_p]),
    "macm_world_status": (c_int, [c_void_p, POINTER(c_int32), c_void_p]),
    "macm_world_counters": (c_int, [c_void_p, POINTER(c_int64), c_void_p]),
    "macm_world_reset_counters": (c_int, [c_void_p, c_void_p]),
    "macm_world_reward_sums": (c_int, [c_void_p, c_void_p, POINTER(c_double), c_void_p]),
    "macm_world_spilled": (c_int, [c_void_p, POINTER(c_int64), c_void_p]),
    "macm_world_set_debug": (c_int, [c_void_p, c_int32]),
    "macm_tdm_config_default": (c_int, [POINTER(MacmTdmConfig)]),
    "macm_tdm_create": (c_int, [POINTER(MacmTdmConfig), c_int32, c_int32, POINTER(c_void_p)]),
    "macm_tdm_destroy": (c_int, [c_void_p]),
    "macm_tdm_reset": (c_int, [c_void_p, c_uint64, c_int64, POINTER(MacmTdmOutputs), c_void_p]),
    "macm_tdm_place": (c_int, [c_void_p, c_void_p, c_void_p, POINTER(MacmTdmOutputs), c_void_p]),
    "macm_tdm_reset_envs": (c_int, [c_void_p, c_void_p, POINTER(MacmTdmOutputs), c_void_p]),
    "macm_tdm_step": (c_int, [c_void_p, c_void_p, POINTER(MacmTdmOutputs), c_void_p]),
    "macm_tdm_rollout": (c_int, [c_void_p, c_void_p, c_int, POINTER(MacmTdmOutputs), c_void_p]),
    "macm_tdm_rollout_bots": (c_int, [c_void_p, c_void_p, c_int, POINTER(MacmTdmOutputs), c_void_p]),
    "macm_tdm_rollout_traj": (c_int, [c_void_p, c_void_p, c_int, POINTER(MacmTdmOutputs), c_void_p]),
    "macm_tdm_rollout_bots_traj": (c_int, [c_void_p, c_void_p, c_int, POINTER(MacmTdmOutputs), c_void_p]),
    "macm_tdm_observe": (c_int, [c_void_p, POINTER(MacmTdmOutputs), c_void_p]),
    "macm_tdm_get_state": (c_int, [c_void_p, POINTER(MacmTdmState), c_void_p]),
    "macm_tdm_set_state": (c_int, [c_void_p, POINTER(MacmTdmState), c_void_p]),
    "macm_tdm_status": (c_int, [c_void_p, POINTER(c_int32), c_void_p]),
    "macm_tdm_counters": (c_int, [c_void_p, POINTER(c_int64), c_void_p]),
    "macm_tdm_spilled": (c_int, [c_void_p, POINTER(c_int64), c_void_p]),
    "macm_tdm_launch_flags": (c_int, [c_void_p]),
    "macm_tdm_reserve": (c_int, [c_void_p, c_int32, c_void_p]),
    "macm_tdm_set_debug": (c_int, [c_void_p, c_int32]),
    "macm_bots_flock": (c_int, [c_void_p, c_int32, c_int32, c_int64, c_void_p, c_void_p]),
    "macm_bots_combat": (c_int, [c_void_p, c_void_p, c_int32, c_int32, c_int64, c_void_p, c_void_p]),
}

_lib = None


def lib():
    """Load libmacm_hip.so (after torch, so the HIP runtime torch loaded is reused)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MacmLibraryError(
            f"{LIB_PATH} not found: build it with `python __graft_entry__.py build` "
            "(no CPU fallback exists for the product path)")
    try:
        import torch  # noqa: F401  (dedupes libamdhip64.so.7 with torch's copy)
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    try:
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:
        raise MacmLibraryError(f"failed to load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(code: int, fn: str) -> None:
    if code != 0:
        msg = lib().macm_last_error()
        msg = msg.decode() if msg else ""
        if code == E_OVERFLOW:
            raise MacmOverflowError(code, fn, msg)
        if code == E_INVALID and fn.endswith(("_step", "_rollout", "_rollout_traj")) and "action space" in msg:
            raise MacmInvalidActionError(code, fn, msg)
        raise MacmError(code, fn, msg)
