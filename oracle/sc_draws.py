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


# ---- normal / sinusoidal demand (demands_generator.py:38-89) ---------------------------
# Restated from the reference: per product a model (kind, lo, hi, std, peaks, minavg,
# maxavg, perturb_norm). The device samples the integer each model ends as from the same
# Philox word as the uniform draw (word j = (t * R + r) * P + p, stream 2):
#   normal       lo + #{k : thr[k] <= u},   thr[k] = floor(P(rint(clip(mean + X)) <= lo + k) * 2^32)
#   sine/normal  the same per period t with mean b_t
#   sine/uniform rint(clip(b_t + jj)),  jj = int(-3 std) + floor(u * n / 2^32),
#                n = int(3 std + 1) - int(-3 std)  (randint truncates float bounds)
# b_t = minavg + (maxavg - minavg) / 2 * (1 + sin(peaks * 2 pi * t / horizon)) in NumPy.
import math  # noqa: E402


def _model_kind(m):
    if m.get("sen_peaks") is None:
        return "uniform" if m.get("std") is None else "normal"
    return "sine_normal" if m.get("perturb_norm", False) else "sine_uniform"


def sine_base(m, horizon):
    half = (m["maxavg"] - m["minavg"]) / 2
    arg = m["sen_peaks"] * 2 * np.pi / horizon
    return np.array([m["minavg"] + half * (1 + np.sin(arg * t)) for t in range(horizon + 1)], dtype=np.float64)


def _cdf_threshold(v, b, std, lo, hi):
    if std == 0:
        cdf = 1.0 if v >= float(np.rint(np.clip(b, lo, hi))) else 0.0
    else:
        cdf = 0.5 * math.erfc(-((v + 0.5 - b) / std) / math.sqrt(2.0))
    t = cdf * 4294967296.0
    return 0xFFFFFFFF if t >= 4294967295.0 else int(t)


def normal_thresholds(m, horizon):
    lo, hi = m["lo"], m["hi"]
    std = 0 if m.get("std") is None else float(m["std"])
    means = [(hi + lo) / 2] if _model_kind(m) == "normal" else list(sine_base(m, horizon))
    return np.array([[_cdf_threshold(lo + k, float(b), std, lo, hi) for k in range(hi - lo)] for b in means],
                    dtype=np.uint32)


def sc_demand_table_models(seed, env_id, episode, T, R, P, models):
    """customer_demands [T+1, R, P] for per-product models (dicts with lo, hi, std,
    sen_peaks, minavg, maxavg, perturb_norm)."""
    words = draw_words(seed, [env_id], episode, (T + 1) * R * P, STREAM_SC_DEMAND)[0].reshape(T + 1, R, P)
    out = np.zeros((T + 1, R, P), dtype=np.int64)
    for p, m in enumerate(models):
        kind, lo, hi = _model_kind(m), m["lo"], m["hi"]
        w = words[:, :, p].astype(np.uint64)
        if kind == "uniform":
            out[:, :, p] = uniform_from_words(words[:, :, p], lo, hi)
        elif kind in ("normal", "sine_normal"):
            thr = normal_thresholds(m, T)
            for t in range(T + 1):
                row = thr[0] if kind == "normal" else thr[t]
                out[t, :, p] = lo + np.searchsorted(row, words[t, :, p], side="right")
        else:
            std = 0 if m.get("std") is None else m["std"]
            plo = int(-3 * std)
            n = int(3 * std + 1) - plo
            jj = plo + ((w * np.uint64(n)) >> np.uint64(32)).astype(np.int64)
            b = sine_base(m, T)[:, None]
            out[:, :, p] = np.rint(np.clip(b + jj, lo, hi)).astype(np.int64)
    return out
