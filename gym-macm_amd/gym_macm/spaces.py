"""Action/observation spaces for the drop-in API.

When gym is importable its spaces are used (the reference builds gym.spaces,
mvmnt.py:142-158). gym is absent in this image, so the fallback below implements
the same constructors and gym 0.21 `contains` semantics the reference's
`assert self.action_space.contains(actions)` (mvmnt.py:94) relies on.
"""
import numpy as np

try:  # pragma: no cover - exercised only where gym is installed
    from gym.spaces import Box, Dict, Discrete, MultiDiscrete, Tuple  # noqa: F401
except Exception:

    class Space(object):
        pass

    class Discrete(Space):
        def __init__(self, n):
            self.n = n

        def contains(self, x):
            return isinstance(x, (int, np.integer)) and 0 <= int(x) < self.n

    class Box(Space):
        def __init__(self, low, high, dtype=np.float32):
            self.dtype = np.dtype(dtype)
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
            x = np.asarray(x)
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
            return all(k in x and s.contains(x[k]) for k, s in self.spaces.items())
