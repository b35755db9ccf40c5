"""gym_macm — MI355X-native drop-in for siyarvurucu/gym-macm's cm-flock-v0 hot path.

Registration mirrors the reference (gym_macm/__init__.py:3-16). gym is optional:
when it is importable the three ids are registered with it, so
``gym.make('gym_macm:cm-flock-v0', n_agents=[N], ...)`` works unchanged; without
gym, :func:`make` resolves the same ids.

Throughput API: :class:`gym_macm.vec.FlockVec` (E envs x N agents, tensors on the GPU).
Drop-in dict API: :class:`gym_macm.envs.Flock` (one env, reference dict surface).
"""
from __future__ import annotations

ENV_IDS = {
    "cm-flock-v0": "gym_macm.envs:Flock",
    "cm-tdm-v0": "gym_macm.envs:TDM",
    "cm-ctdm-v0": "gym_macm.envs:ControlledTDM",
}

try:  # pragma: no cover - gym is not installed in this image
    from gym.envs.registration import register as _register

    for _id, _ep in ENV_IDS.items():
        _register(id=_id, entry_point=_ep)
except Exception:
    pass


def make(env_id: str, **kwargs):
    """gym.make equivalent for the registered ids (accepts 'gym_macm:cm-flock-v0')."""
    import importlib

    key = env_id.split(":", 1)[1] if ":" in env_id else env_id
    if key not in ENV_IDS:
        raise KeyError(f"unknown env id {env_id!r}; known: {sorted(ENV_IDS)}")
    mod, cls = ENV_IDS[key].split(":")
    return getattr(importlib.import_module(mod), cls)(**kwargs)
