"""The reference's scripted actors (test_scripts/bots.py) as device kernels.

    act = flock_actions(vec.obs)                 # bots.flock for every agent, uint8 [E, N, 3]
    act = combat_actions(w.obs, w.mask)          # bots.combat for every agent, uint8 [E, N, 4]

Both read the observation tensors a step wrote and launch on the current stream,
so `step -> bots -> step` never leaves HBM. With float64 observations the
decisions equal the reference bots' on the same observations (bots.py:3-16, 37-61).
"""
from __future__ import annotations

import ctypes

import torch

from . import _abi


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check_obs(obs):
    if obs.device.type != "cuda" or not obs.is_contiguous():
        raise ValueError("obs must be a contiguous tensor on a GPU")
    if obs.dtype not in (torch.float32, torch.float64):
        raise ValueError("obs must be float32 or float64")


def flock_actions(obs: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """bots.flock on Flock observations [..., 4] (polar) or [..., 6] (cartesian)."""
    _check_obs(obs)
    od = obs.shape[-1]
    rows = obs.numel() // od
    if out is None:
        out = torch.empty(tuple(obs.shape[:-1]) + (3,), dtype=torch.uint8, device=obs.device)
    L = _abi.lib()
    _abi.check(L.macm_bots_flock(ctypes.c_void_p(obs.data_ptr()), 1 if obs.dtype == torch.float64 else 0, od,
                                 rows, ctypes.c_void_p(out.data_ptr()), _stream(obs)), "macm_bots_flock")
    return out


def combat_actions(obs: torch.Tensor, mask: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """bots.combat on TDM observations [E, N, N-1, 4] with mask [E, N, N-1]."""
    _check_obs(obs)
    if obs.dim() != 4 or obs.shape[-1] != 4 or tuple(mask.shape) != tuple(obs.shape[:-1]):
        raise ValueError("expected obs [E, N, N-1, 4] and mask [E, N, N-1]")
    if mask.dtype != torch.uint8 or not mask.is_contiguous() or mask.device != obs.device:
        raise ValueError("mask must be a contiguous uint8 tensor on the obs device")
    E, N = obs.shape[0], obs.shape[1]
    if out is None:
        out = torch.empty((E, N, 4), dtype=torch.uint8, device=obs.device)
    L = _abi.lib()
    _abi.check(L.macm_bots_combat(ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(mask.data_ptr()),
                                  1 if obs.dtype == torch.float64 else 0, N, E * N,
                                  ctypes.c_void_p(out.data_ptr()), _stream(obs)), "macm_bots_combat")
    return out
