"""Space descriptors.

The reference declares spaces with gym.spaces (SupplyChainEnv: Box(-1, 1),
supplychain_env.py:625-626) and leaves BeerGameEnv's commented out
(beergame_env.py:62-64). gym/gymnasium are optional here: when one is importable its
classes are used, otherwise these minimal shape/bounds holders stand in. Spaces are
metadata only — no env in this package samples from them on the step path.
"""
import numpy as np

try:  # prefer the real thing when present
    import gymnasium as _gym  # type: ignore
except ImportError:  # pragma: no cover - depends on the image
    try:
        import gym as _gym  # type: ignore
    except ImportError:
        _gym = None


class _Box:
    def __init__(self, low, high, shape, dtype):
        self.dtype = np.dtype(dtype)
        self.shape = tuple(shape)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


def Box(low, high, shape, dtype=np.float32):
    if _gym is not None:
        return _gym.spaces.Box(low=low, high=high, shape=tuple(shape), dtype=dtype)
    return _Box(low, high, shape, dtype)
