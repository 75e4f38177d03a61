"""Gymnasium spaces if installed, else a minimal Box with the same attributes.

The reference declares `spaces.Box(-inf, inf, (79,), float32)` and `Box(-1, 1, (2,), float32)`
(src/rl/envs/ackermann_env.py:95-108). gymnasium is not installed in this image.
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium exists
    from gymnasium import spaces as _gs
    Box = _gs.Box
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
            self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()
            self._rng = np.random.default_rng(seed)

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return self._rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


def observation_space():
    return Box(low=-np.inf, high=np.inf, shape=(79,), dtype=np.float32)


def action_space():
    return Box(low=-1.0, high=1.0, shape=(2,), dtype=np.float32)
