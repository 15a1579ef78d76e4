"""Observation/action spaces (smart_nanogrid_environment.py:90-120).

Uses gymnasium.spaces.Box or gym.spaces.Box when one of them is importable, so SB3
sees the class it expects; otherwise a minimal Box with the same attributes.
"""
import numpy as np

try:
    from gymnasium.spaces import Box as _Box   # pragma: no cover - not installed in the image
except Exception:
    try:
        from gym.spaces import Box as _Box     # pragma: no cover
    except Exception:
        _Box = None


class _MiniBox:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low)
        self.shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()
        self._rng = np.random.default_rng()

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


Box = _Box if _Box is not None else _MiniBox


def make_spaces(settings):
    n = settings.number_of_chargers
    obs_low = np.zeros(settings.obs_dim, dtype=np.float32)
    obs_high = np.ones(settings.obs_dim, dtype=np.float32)
    observation_space = Box(low=obs_low, high=obs_high, dtype=np.float32)
    if settings.bess:
        if settings.v2x:
            low = np.ones(n + 1, dtype=np.float32) * (-1)
        else:
            low = np.insert(np.zeros(n, dtype=np.float32), n, -1)
        high = np.ones(n + 1, dtype=np.float32)
        action_space = Box(low=low, high=high, shape=(n + 1,), dtype=np.float32)
    else:
        action_space = Box(low=-1 if settings.v2x else 0, high=1, shape=(n,), dtype=np.float32)
    return observation_space, action_space
