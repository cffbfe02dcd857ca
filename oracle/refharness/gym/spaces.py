"""Inert shape holders standing in for gym.spaces (see gym/__init__.py)."""
import numpy as np


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        self.shape = tuple(shape) if shape is not None else np.shape(low)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def seed(self, seed=None):
        return [seed]

    def sample(self):
        raise RuntimeError("stub Box.sample(): golden vectors use explicit actions only")


class MultiDiscrete:
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec)
        self.shape = self.nvec.shape

    def seed(self, seed=None):
        return [seed]

    def sample(self):
        raise RuntimeError("stub MultiDiscrete.sample(): golden vectors use explicit actions only")


class Discrete:
    def __init__(self, n):
        self.n = n
        self.shape = ()
