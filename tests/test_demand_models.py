"""Normal / sinusoidal demand models (demands_generator.py:38-89) as the device draws them.

* The host tables the kernels read (envs/demand.py) equal the oracle's restatement
  (oracle/sc_draws.py) — thresholds and sinusoid bases, bit for bit.
* The distribution those tables define equals the reference generator's: its histograms,
  recorded from the reference itself with RandomState (tests/golden/demand_models.npz,
  oracle/gen_golden_demand.py), pass a chi-square test against the exact pmf of the
  device's draw (inverse CDF of rint(clip(b + N(0, std))) / uniform integer perturbation).
* The oracle's Philox draws of every model follow that pmf (the word -> value mapping).
"""
import json
import os

import numpy as np
import pytest
from scipy import stats

from conftest import REPO
from oracle import sc_draws

GOLDEN = os.path.join(REPO, "tests", "golden", "demand_models.npz")


def _load():
    z = dict(np.load(GOLDEN, allow_pickle=False))
    return z, json.loads(str(z.pop("meta")))


def _model(kw):
    return dict(lo=kw["minv"], hi=kw["maxv"], std=kw.get("std"), sen_peaks=kw.get("sen_peaks"),
                minavg=kw.get("minavg"), maxavg=kw.get("maxavg"), perturb_norm=kw.get("perturb_norm", True))


def _pmf(m, horizon, period):
    """Exact pmf over lo..hi of the device's draw at `period`."""
    lo, hi = m["lo"], m["hi"]
    kind = sc_draws._model_kind(m)
    if kind in ("normal", "sine_normal"):
        thr = sc_draws.normal_thresholds(m, horizon)
        row = thr[0] if kind == "normal" else thr[period]
        cdf = np.concatenate([row.astype(np.float64), [2.0 ** 32]]) / 2.0 ** 32
        return np.diff(np.concatenate([[0.0], cdf]))
    std = 0 if m["std"] is None else m["std"]
    plo = int(-3 * std)
    n = int(3 * std + 1) - plo
    b = sc_draws.sine_base(m, horizon)[period]
    pmf = np.zeros(hi - lo + 1)
    for j in range(plo, plo + n):
        pmf[int(np.rint(np.clip(b + j, lo, hi))) - lo] += 1.0 / n
    return pmf


def _chi2_pvalue(counts, pmf):
    """Chi-square goodness of fit; bins with fewer than 5 expected draws pooled into one."""
    counts = np.asarray(counts, dtype=np.float64)
    n = counts.sum()
    exp = pmf / pmf.sum() * n
    keep = exp >= 5
    obs, ex = list(counts[keep]), list(exp[keep])
    if (~keep).any():
        obs.append(counts[~keep].sum())
        ex.append(exp[~keep].sum())
    obs, ex = np.array(obs), np.array(ex)
    if ex[-1] < 5 and len(ex) > 1:  # a sparse pooled tail joins the previous bin
        obs[-2] += obs[-1]
        ex[-2] += ex[-1]
        obs, ex = obs[:-1], ex[:-1]
    if len(obs) == 1:
        return 1.0
    return stats.chisquare(obs, ex * (obs.sum() / ex.sum())).pvalue


def test_golden_present():
    z, meta = _load()
    assert set(meta["models"]) == {"normal", "normal_narrow", "seasonal", "sine_normal", "sine_uniform", "sine_flat"}


def test_device_tables_equal_oracle():
    from gym_supplychain_amd.envs import demand
    _, meta = _load()
    T = meta["horizon"]
    for name, kw in meta["models"].items():
        m = _model(kw)
        dm = demand.DemandModel(m["lo"], m["hi"], m["std"], m["sen_peaks"], m["minavg"], m["maxavg"], m["perturb_norm"])
        if dm.kind in (demand.NORMAL, demand.SINE_NORMAL):
            assert np.array_equal(dm.thresholds(T), sc_draws.normal_thresholds(m, T)), name
        if dm.kind in (demand.SINE_NORMAL, demand.SINE_UNIFORM):
            assert np.array_equal(dm.sine_base(T), sc_draws.sine_base(m, T)), name


@pytest.mark.parametrize("name", ["normal", "normal_narrow", "seasonal", "sine_normal", "sine_uniform", "sine_flat"])
def test_distribution_matches_reference_generator(name):
    z, meta = _load()
    m = _model(meta["models"][name])
    periods = [0] if m["sen_peaks"] is None else meta["periods"]
    for i, t in enumerate(periods):
        counts = z[name][i]
        pmf = _pmf(m, meta["horizon"], t)
        if m["sen_peaks"] is not None and (m["std"] in (None, 0)):
            assert np.array_equal(counts > 0, pmf > 0), (name, t)   # deterministic sinusoid
            continue
        p = _chi2_pvalue(counts, pmf)
        assert p > 1e-6, (name, t, p)


def test_oracle_draws_follow_the_model():
    """The oracle's word -> value mapping over many (env, episode) draws against the pmf."""
    _, meta = _load()
    T = 12
    for name in ("normal", "sine_normal", "sine_uniform"):
        m = _model(meta["models"][name])
        draws = np.stack([sc_draws.sc_demand_table_models(5, e, 0, T, 1, 1, [m])[:, 0, 0] for e in range(3000)])
        for t in (0, 7):
            counts = np.bincount(draws[:, t] - m["lo"], minlength=m["hi"] - m["lo"] + 1)
            assert _chi2_pvalue(counts, _pmf(m, T, t)) > 1e-6, (name, t)
