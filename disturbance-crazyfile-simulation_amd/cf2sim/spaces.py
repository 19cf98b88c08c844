"""Minimal gym-compatible spaces (gym is not a dependency; when it is importable its Box is used).

Mirrors the spaces DroneBaseEnv declares (envs/base.py:139-148): observations
Box(-1000, 1000, (34|42,), float32), actions Box(-1, 1, (4,), float32).
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - gym is absent in this image
    from gym.spaces import Box as _GymBox  # type: ignore
except Exception:  # noqa: BLE001
    _GymBox = None


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.dtype = np.dtype(dtype)
        if shape is None:
            low = np.asarray(low, dtype=self.dtype)
            shape = low.shape
        self.shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()
        self.bounded_below = np.isfinite(self.low)
        self.bounded_above = np.isfinite(self.high)
        self.np_random = np.random.default_rng(seed)

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        return self.np_random.uniform(self.low, self.high, size=self.shape).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    def __eq__(self, other):
        return (isinstance(other, Box) and self.shape == other.shape and np.allclose(self.low, other.low)
                and np.allclose(self.high, other.high))


def make_box(low, high, shape=None, dtype=np.float32):
    if _GymBox is not None:  # pragma: no cover
        return _GymBox(low, high, shape=shape, dtype=dtype)
    return Box(low, high, shape=shape, dtype=dtype)
