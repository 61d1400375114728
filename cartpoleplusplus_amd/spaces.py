"""Minimal stand-ins for the two gym spaces the reference uses (gym is not
installed here; bullet_cartpole.py:91-94 and :140-141 only construct `Discrete`
and `Box` and callers read `.n`, `.shape`, `.low`, `.high`, `.sample()`).
If gym or gymnasium is importable, their classes are used instead."""
import numpy as np

try:  # pragma: no cover - depends on the environment
    from gym import Env, spaces as _gs  # type: ignore
    Discrete, Box = _gs.Discrete, _gs.Box
except Exception:  # noqa: BLE001
    try:  # pragma: no cover
        from gymnasium import Env, spaces as _gs  # type: ignore
        Discrete, Box = _gs.Discrete, _gs.Box
    except Exception:  # noqa: BLE001
        class Env:
            """Base class placeholder with the old gym method names."""

            metadata = {}

        class Discrete:
            def __init__(self, n):
                self.n = int(n)
                self.shape = ()
                self.dtype = np.int64

            def sample(self):
                return int(np.random.randint(self.n))

            def contains(self, x):
                return isinstance(x, (int, np.integer)) and 0 <= x < self.n

            def __repr__(self):
                return f"Discrete({self.n})"

        class Box:
            def __init__(self, low, high, shape=None, dtype=np.float32):
                self.shape = tuple(shape) if shape is not None else np.shape(low)
                self.dtype = dtype
                self.low = np.full(self.shape, low, dtype=dtype) if np.isscalar(low) else np.asarray(low, dtype)
                self.high = np.full(self.shape, high, dtype=dtype) if np.isscalar(high) else np.asarray(high, dtype)

            def sample(self):
                lo = np.maximum(self.low, -1e30)
                hi = np.minimum(self.high, 1e30)
                return np.random.uniform(lo, hi, self.shape).astype(self.dtype)

            def contains(self, x):
                x = np.asarray(x)
                return x.shape == self.shape and np.all(x >= self.low) and np.all(x <= self.high)

            def __repr__(self):
                return f"Box{self.shape}"
