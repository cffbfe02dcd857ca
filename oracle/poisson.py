"""Poisson(lambda) inverse-CDF on uint32 thresholds — TEST INFRASTRUCTURE ONLY.

Integer-only inversion so the host oracle and the HIP kernel draw bit-identical
demands from the same Philox words:

    thr[k] = min(floor(CDF(k) * 2**32), 2**32 - 1),  k = 0 .. K-1,
    the table ends at the first k whose threshold saturates;
    sample(u) = #{k : thr[k] <= u}   (u a uint32 Philox word).

P(sample == k) = (thr[k] - thr[k-1]) / 2**32, i.e. the Poisson pmf to 2**-32.
The float64 recurrence below (exp(-lam), p *= lam / (k+1), c += p) is the same
sequence of IEEE operations as scg_poisson_table() in the product library, so the
two tables are identical (checked in tests/test_oracle_beergame.py).
"""
import math

import numpy as np

MAX_TABLE = 256


def poisson_thresholds(lam, max_len=MAX_TABLE):
    lam = float(lam)
    if not (lam >= 0.0) or math.isinf(lam):
        raise ValueError(f"poisson lambda must be a finite value >= 0, got {lam}")
    p = math.exp(-lam)
    c = p
    thr = []
    for k in range(max_len):
        t = c * 4294967296.0
        t = 0xFFFFFFFF if t >= 4294967295.0 else int(t)
        thr.append(t)
        if t == 0xFFFFFFFF:
            return np.asarray(thr, dtype=np.uint32)
        p = p * lam / (k + 1)
        c = c + p
    raise ValueError(f"poisson lambda {lam} needs more than {max_len} CDF thresholds")


def poisson_invert(words, thr):
    """words: uint32 array; thr: threshold table. Returns int32 draws."""
    words = np.asarray(words, dtype=np.uint32)
    thr = np.asarray(thr, dtype=np.uint32)
    return np.searchsorted(thr, words, side="right").astype(np.int32)
