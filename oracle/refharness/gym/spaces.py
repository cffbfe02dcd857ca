"""Stand-ins for gym 0.21's Box / MultiDiscrete / Discrete (build container only; see
gym/__init__.py): shape holders whose seed()/sample() restate gym 0.21.0 (Space.seed via
utils/seeding.np_random; Box.sample = uniform(low, high) over the bounded dims, cast to the
dtype; MultiDiscrete.sample = floor(random_sample * nvec)), so the reference's episode-reward
pins, which sample actions, can be re-run here (oracle/gen_golden_pins.py)."""
import numpy as np

from .utils import seeding


class Space:
    _np_random = None

    @property
    def np_random(self):
        if self._np_random is None:
            self.seed()
        return self._np_random

    def seed(self, seed=None):
        self._np_random, seed = seeding.np_random(seed)
        return [seed]


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        self.shape = tuple(shape) if shape is not None else np.shape(low)
        self.low = np.full(self.shape, low, dtype=self.dtype) if np.isscalar(low) else np.asarray(low, self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype) if np.isscalar(high) else np.asarray(high, self.dtype)

    def sample(self):
        below, above = -np.inf < self.low, np.inf > self.high
        high = self.high if self.dtype.kind == "f" else self.high.astype("int64") + 1
        x = np.empty(self.shape)
        both = below & above
        x[~below & ~above] = self.np_random.normal(size=int((~below & ~above).sum()))
        x[below & ~above] = self.np_random.exponential(size=int((below & ~above).sum())) + self.low[below & ~above]
        x[~below & above] = -self.np_random.exponential(size=int((~below & above).sum())) + self.high[~below & above]
        x[both] = self.np_random.uniform(low=self.low[both], high=high[both], size=int(both.sum()))
        if self.dtype.kind == "i":
            x = np.floor(x)
        return x.astype(self.dtype)


class MultiDiscrete(Space):
    def __init__(self, nvec, dtype=np.int64):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
        self.dtype = np.dtype(dtype)

    def sample(self):
        return (self.np_random.random_sample(self.nvec.shape) * self.nvec).astype(self.dtype)


class Discrete(Space):
    def __init__(self, n):
        self.n = n
        self.shape = ()

    def sample(self):
        return self.np_random.randint(self.n)
