"""Stand-in for gym 0.21's gym/utils/seeding.py (build container only; see gym/__init__.py).

gym 0.21 seeds a space's RandomState from sha512 of the decimal seed: the first 8 digest
bytes, read as little-endian uint32 words, form a bigint that is split back into uint32
words for RandomState.seed. Restated from gym 0.21.0's published seeding.py so the
reference's action_space.sample() calls draw what its tests were pinned with.
"""
import hashlib
import os
import struct

import numpy as np


def _words_to_int(data):
    data = data + b"\0" * (4 - len(data) % 4)
    n = len(data) // 4
    return sum(v * 2 ** (32 * i) for i, v in enumerate(struct.unpack(f"{n}I", data)))


def _int_to_words(value):
    if value == 0:
        return [0]
    words = []
    while value:
        value, low = divmod(value, 2 ** 32)
        words.append(low)
    return words


def create_seed(a=None, max_bytes=8):
    if a is None:
        return _words_to_int(os.urandom(max_bytes))
    if isinstance(a, str):
        b = a.encode("utf8")
        return _words_to_int((b + hashlib.sha512(b).digest())[:max_bytes])
    return int(a) % 2 ** (8 * max_bytes)


def hash_seed(seed=None, max_bytes=8):
    if seed is None:
        seed = create_seed(max_bytes=max_bytes)
    return _words_to_int(hashlib.sha512(str(seed).encode("utf8")).digest()[:max_bytes])


def np_random(seed=None):
    seed = create_seed(seed)
    rng = np.random.RandomState()
    rng.seed(_int_to_words(hash_seed(seed)))
    return rng, seed
