"""Minimal `gym` stand-in used ONLY by make_golden.py to import the reference env.

gym is not installed in this image (and no network). The reference touches gym in
three places: `gym.Env` as a base class (mvmnt.py:27), `gym.spaces` constructors +
`Dict.contains` (mvmnt.py:94,142-158) and `gym.envs.registration.register`
(gym_macm/__init__.py:1-16). This module provides exactly those with gym 0.21
semantics for `contains` (Dict: same keys, each sub-space contains its value;
MultiDiscrete: shape match and 0 <= x < nvec; Box: castable dtype, shape, bounds).
"""
import sys
import types

import numpy as np


class Env(object):
    pass


class Space(object):
    pass


class Discrete(Space):
    def __init__(self, n):
        self.n = n


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        if shape is not None:  # gym 0.21: scalar bounds broadcast to `shape`
            low = np.full(shape, low) if np.isscalar(low) else low
            high = np.full(shape, high) if np.isscalar(high) else high
        self.low = np.asarray(low).astype(self.dtype)
        self.high = np.asarray(high).astype(self.dtype)
        self.shape = self.low.shape

    def contains(self, x):
        if not isinstance(x, np.ndarray):
            x = np.asarray(x, dtype=self.dtype)
        return bool(np.can_cast(x.dtype, self.dtype) and x.shape == self.shape
                    and np.all(x >= self.low) and np.all(x <= self.high))


class MultiDiscrete(Space):
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape

    def contains(self, x):
        if isinstance(x, list):
            x = np.array(x)
        return x.shape == self.shape and bool((0 <= x).all()) and bool((x < self.nvec).all())


class Tuple(Space):
    def __init__(self, spaces):
        self.spaces = tuple(spaces)


class Dict(Space):
    def __init__(self, spaces):
        self.spaces = dict(spaces)

    def contains(self, x):
        if not isinstance(x, dict) or len(x) != len(self.spaces):
            return False
        for k, space in self.spaces.items():
            if k not in x:
                return False
            if not space.contains(x[k]):
                return False
        return True


_registry = {}


def register(id, entry_point, **kwargs):
    _registry[id] = entry_point


def install():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")
    envs = types.ModuleType("gym.envs")
    registration = types.ModuleType("gym.envs.registration")
    for cls in (Space, Discrete, Box, MultiDiscrete, Tuple, Dict):
        setattr(spaces, cls.__name__, cls)
    registration.register = register
    envs.registration = registration
    gym.Env = Env
    gym.spaces = spaces
    gym.envs = envs
    sys.modules.update({"gym": gym, "gym.spaces": spaces, "gym.envs": envs,
                        "gym.envs.registration": registration})
