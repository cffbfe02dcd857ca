"""gym spaces with the sampling the reference's tests were pinned with (gym <= 0.21).

The reference declares SupplyChainEnv's spaces with gym.spaces.Box(-1, 1)
(supplychain_env.py:625-626), BeerGameEnv2's with MultiDiscrete (beergame2_env.py:27-28),
and SupplyChainEnv.seed() calls action_space.seed(0) (:811-813). Its episode-reward pins
(test_Nperstage.py:23-53, test_multiproduct_2perstage.py:221-309) come from
`action_space.sample()` under gym 0.21, whose Space seeding is

    seed % 2**64 -> sha512(str(seed))[:8] as a little-endian bigint -> uint32 list
    -> RandomState.seed(list)                                 (gym/utils/seeding.py, 0.21)

and whose Box.sample draws `uniform(low, high)` (float64) for bounded dims and casts to
the Box dtype (gym/spaces/box.py, 0.21). Later gym versions use PCG64 and give other
actions, so these classes restate the 0.21 algorithm (published code of gym 0.21.0, not
part of /root/reference) and are what the package's envs expose. When `gym` is
importable they subclass its classes, so `isinstance(space, gym.spaces.Box)` holds.
Spaces are host metadata: no env here samples from them on the step path.
"""
import hashlib
import os
import struct

import numpy as np

try:  # the reference's gym (old API); gymnasium's Env/spaces have a different contract
    import gym as _gym  # type: ignore
except ImportError:  # pragma: no cover - depends on the image (absent here and on the GPU box)
    _gym = None


# ---- gym 0.21 seeding (gym/utils/seeding.py) ----------------------------------------------
def _bigint_from_bytes(b):
    pad = 4 - len(b) % 4  # 0.21 pads a full word when already aligned (adds a zero word)
    b = b + b"\0" * pad
    words = struct.unpack(f"{len(b) // 4}I", b)
    return sum(w << (32 * i) for i, w in enumerate(words))


def _int_list_from_bigint(x):
    if x < 0:
        raise ValueError(f"seed must be non-negative, got {x}")
    if x == 0:
        return [0]
    out = []
    while x > 0:
        x, mod = divmod(x, 2 ** 32)
        out.append(mod)
    return out


def create_seed(a=None, max_bytes=8):
    if a is None:
        return _bigint_from_bytes(os.urandom(max_bytes))
    if isinstance(a, str):
        a = a.encode("utf8")
        a += hashlib.sha512(a).digest()
        return _bigint_from_bytes(a[:max_bytes])
    if isinstance(a, (int, np.integer)):
        return int(a) % 2 ** (8 * max_bytes)
    raise TypeError(f"invalid seed type {type(a)}")


def hash_seed(seed=None, max_bytes=8):
    if seed is None:
        seed = create_seed(max_bytes=max_bytes)
    digest = hashlib.sha512(str(seed).encode("utf8")).digest()
    return _bigint_from_bytes(digest[:max_bytes])


def np_random(seed=None):
    """(RandomState, seed) as gym 0.21's seeding.np_random."""
    if seed is not None and not (isinstance(seed, (int, np.integer)) and seed >= 0):
        raise ValueError(f"Seed must be a non-negative integer or omitted, not {seed!r}")
    seed = create_seed(seed)
    rng = np.random.RandomState()
    rng.seed(_int_list_from_bigint(hash_seed(seed)))
    return rng, seed


# ---- spaces -------------------------------------------------------------------------------
class _Space21:
    """Space.seed / np_random of gym 0.21: lazily seeded from os.urandom."""

    _rng = None

    @property
    def np_random(self):
        if self._rng is None:
            self.seed()
        return self._rng

    def seed(self, seed=None):
        self._rng, seed = np_random(seed)
        return [seed]


_BoxBase = (_gym.spaces.Box,) if _gym is not None else ()
_MDBase = (_gym.spaces.MultiDiscrete,) if _gym is not None else ()


class Box(_Space21, *_BoxBase):
    """Box(low, high, shape, dtype=float32) with gym 0.21 sampling."""

    def __init__(self, low, high, shape=None, dtype=np.float32):
        dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low)
        shape = tuple(int(s) for s in shape)
        if _BoxBase:
            try:
                _BoxBase[0].__init__(self, low=low, high=high, shape=shape, dtype=dtype)
            except Exception:  # pragma: no cover - an incompatible gym; our fields below suffice
                pass
        self.dtype = dtype
        self.shape = self._shape = shape
        self.low = np.full(shape, low, dtype=np.float64).astype(dtype) if np.isscalar(low) \
            else np.asarray(low).astype(dtype)
        self.high = np.full(shape, high, dtype=np.float64).astype(dtype) if np.isscalar(high) \
            else np.asarray(high).astype(dtype)
        self.bounded_below = -np.inf < self.low
        self.bounded_above = np.inf > self.high
        self._rng = None

    def is_bounded(self, manner="both"):
        below, above = bool(np.all(self.bounded_below)), bool(np.all(self.bounded_above))
        return {"both": below and above, "below": below, "above": above}[manner]

    def sample(self):
        """gym 0.21 Box.sample: normal / exponential draws for unbounded dims, uniform for
        bounded ones (in that order, each drawing only as many values as it has dims),
        floor for integer boxes, cast to dtype."""
        rng = self.np_random
        high = self.high if self.dtype.kind == "f" else self.high.astype("int64") + 1
        out = np.empty(self.shape)
        unb = ~self.bounded_below & ~self.bounded_above
        upp = ~self.bounded_below & self.bounded_above
        low_b = self.bounded_below & ~self.bounded_above
        both = self.bounded_below & self.bounded_above
        out[unb] = rng.normal(size=unb[unb].shape)
        out[low_b] = rng.exponential(size=low_b[low_b].shape) + self.low[low_b]
        out[upp] = -rng.exponential(size=upp[upp].shape) + self.high[upp]
        out[both] = rng.uniform(low=self.low[both], high=high[both], size=both[both].shape)
        if self.dtype.kind == "i":
            out = np.floor(out)
        return out.astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    __contains__ = contains

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    def __eq__(self, other):
        return (isinstance(other, Box) and self.shape == other.shape and np.array_equal(self.low, other.low)
                and np.array_equal(self.high, other.high))

    __hash__ = object.__hash__


class MultiDiscrete(_Space21, *_MDBase):
    """MultiDiscrete(nvec) with gym 0.21 sampling: floor(random_sample * nvec)."""

    def __init__(self, nvec, dtype=np.int64):
        if _MDBase:
            try:
                _MDBase[0].__init__(self, nvec)
            except Exception:  # pragma: no cover
                pass
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.dtype = np.dtype(dtype)
        self.shape = self._shape = self.nvec.shape
        self._rng = None

    def sample(self):
        return (self.np_random.random_sample(self.nvec.shape) * self.nvec).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= 0) and np.all(x < self.nvec))

    __contains__ = contains

    def __repr__(self):
        return f"MultiDiscrete({self.nvec})"

    def __eq__(self, other):
        return isinstance(other, MultiDiscrete) and np.array_equal(self.nvec, other.nvec)

    __hash__ = object.__hash__


# ---- gym.Env base ---------------------------------------------------------------------------
if _gym is not None:
    Env = _gym.Env
else:
    class Env:
        """Stand-in for gym.Env (old API, reset() -> obs, step() -> 4-tuple) when gym is
        absent: the attributes and no-op hooks trainers read."""

        metadata = {"render.modes": []}
        reward_range = (-float("inf"), float("inf"))
        spec = None
        action_space = None
        observation_space = None

        @property
        def unwrapped(self):
            return self

        def seed(self, seed=None):
            return [seed]

        def render(self, mode="human"):
            raise NotImplementedError

        def close(self):
            pass

        def __enter__(self):
            return self

        def __exit__(self, *args):
            self.close()
            return False

        def __str__(self):
            return f"<{type(self).__name__} instance>"
