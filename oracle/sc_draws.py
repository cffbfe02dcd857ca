"""Per-episode random tables of SupplyChainEnv as the device draws them — TEST INFRASTRUCTURE.

The reference draws them at reset with MT19937 RandomState (supplychain_env.py:644-672):
    customer_demands = randint(lo, hi + 1, (T+1, R, P))                   (uniform_data, demands_generator.py:33-36)
    leadtimes        = clip(1 + poisson(avg - 1, (T, n_lt)), 1, max_leadtime)
scgpu draws the same distributions per (env, episode) with Philox4x32-10 instead
(SURVEY §8(f)3): counter (global env id, episode, word // 4, stream), key = seed.
    demand word j = (t * R + r) * P + p, stream 2: lo + floor(u * (hi - lo + 1) / 2**32)
    lead-time word j = t * n_lt + k,    stream 3: clip(1 + Poisson(avg - 1), 1, max)
"""
import numpy as np

from oracle.philox import draw_words
from oracle.poisson import poisson_invert, poisson_thresholds

STREAM_SC_DEMAND = 2
STREAM_SC_LEADTIME = 3


def uniform_from_words(words, lo, hi):
    span = np.uint64(hi - lo + 1)
    return lo + ((words.astype(np.uint64) * span) >> np.uint64(32)).astype(np.int64)


def sc_demand_table(seed, env_id, episode, T, R, P, lo, hi):
    words = draw_words(seed, [env_id], episode, (T + 1) * R * P, STREAM_SC_DEMAND)[0]
    return uniform_from_words(words, lo, hi).reshape(T + 1, R, P)


def sc_leadtime_table(seed, env_id, episode, T, n_lt, avg, max_lt):
    words = draw_words(seed, [env_id], episode, T * n_lt, STREAM_SC_LEADTIME)[0]
    x = 1 + poisson_invert(words, poisson_thresholds(avg - 1)).astype(np.int64)
    return np.clip(x, 1, max_lt).reshape(T, n_lt)
