"""Episode demand models of SupplyChainEnv on the device (demands_generator.py:3-89).

The reference draws a whole episode's demand table at reset() with MT19937 RandomState
(supplychain_env.py:644-661): per product one of

    uniform     randint(lo, hi + 1)                                     uniform_data (:33-36)
    normal      rint(clip(normal((hi + lo) / 2, std), lo, hi))          normal_data (:38-49)
    sinusoidal  rint(clip(b_t + perturbation, lo, hi)),                 senoidal_data (:51-89)
                b_t = minavg + (maxavg - minavg) / 2 * (1 + sin(peaks * 2 pi t / horizon)),
                perturbation normal(0, std) or randint(-3 std, 3 std + 1)

The kernels draw the same distributions per (env, episode, period, retailer, product) from
one Philox4x32-10 word u (the uniform path's word, oracle/sc_draws.py). A normal draw is
sampled by inverting the exact CDF of the integer it ends as — P(rint(clip(b + X)) <= k) =
Phi((k + 0.5 - b) / std) for lo <= k < hi — against a uint32 threshold table built here
once (a count of thresholds <= u, like the Poisson lead times), so no transcendental runs
on the device and host and device draws are bit-identical. The sinusoid's base b_t is
evaluated here with NumPy exactly as the reference writes it and uploaded as float64; a
uniform perturbation j is added on the device and rounded with rint, both exact IEEE
operations.
"""
import math

import numpy as np

UNIFORM, NORMAL, SINE_NORMAL, SINE_UNIFORM = 0, 1, 2, 3
_TWO32 = 4294967296.0


class DemandModel:
    """One product's demand generator (the arguments generate_demand receives, :3-31)."""

    def __init__(self, lo, hi, std=None, sen_peaks=None, minavg=None, maxavg=None, perturb_norm=True):
        self.lo, self.hi = int(lo), int(hi)
        if self.hi <= self.lo:
            raise ValueError(f"demand range ({lo}, {hi}) must have low < high")
        self.std, self.peaks, self.minavg, self.maxavg = std, sen_peaks, minavg, maxavg
        self.perturb_norm = bool(perturb_norm)
        if sen_peaks is None:
            self.kind = UNIFORM if std is None else NORMAL
        else:
            if minavg is None or maxavg is None:
                raise ValueError("sinusoidal demand needs avg_demand_range (minavg, maxavg)")
            self.std = 0 if std is None else std                                    # :30
            self.kind = SINE_NORMAL if self.perturb_norm else SINE_UNIFORM
        if self.kind in (NORMAL, SINE_NORMAL) and not float(self.std) >= 0:
            raise ValueError(f"demand_std must be >= 0, got {std!r}")
        # randint(low=-3 std, high=3 std + 1) truncates float bounds toward zero (:74)
        self.pert_lo = int(-3 * self.std) if self.kind == SINE_UNIFORM else 0
        self.pert_n = int(3 * self.std + 1) - self.pert_lo if self.kind == SINE_UNIFORM else 0
        if self.kind == SINE_UNIFORM and self.pert_n < 1:
            raise ValueError("sinusoidal uniform perturbation needs demand_std >= 0")

    # host tables -------------------------------------------------------------------
    def sine_base(self, horizon):
        """b_t for t = 0..horizon, evaluated as senoidal_data does (:66-86)."""
        curve_range = self.maxavg - self.minavg
        half_curve = curve_range / 2
        sin_arg = self.peaks * 2 * np.pi / horizon
        return np.array([self.minavg + half_curve * (1 + np.sin(sin_arg * period)) for period in range(horizon + 1)],
                        dtype=np.float64)

    def thresholds(self, horizon):
        """uint32 CDF thresholds [rows][hi - lo]: rows = 1 (normal) or horizon + 1 (sinusoid
        with normal perturbation); draw = lo + #{k : thr[row][k] <= u}."""
        if self.kind == NORMAL:
            centres = [(self.hi + self.lo) / 2]                                      # :43
        elif self.kind == SINE_NORMAL:
            centres = list(self.sine_base(horizon))
        else:
            raise ValueError("only normal models use threshold tables")
        out = np.empty((len(centres), self.hi - self.lo), dtype=np.uint32)
        for row, b in enumerate(centres):
            for k in range(self.hi - self.lo):
                out[row, k] = _threshold(self.lo + k, float(b), float(self.std), self.lo, self.hi)
        return out


def _threshold(k, b, std, lo, hi):
    """floor(P(rint(clip(b + X, lo, hi)) <= k) * 2^32), X ~ N(0, std), clamped to 2^32 - 1."""
    if std == 0:
        d = float(np.rint(np.clip(b, lo, hi)))
        cdf = 1.0 if k >= d else 0.0
    else:
        cdf = 0.5 * math.erfc(-((k + 0.5 - b) / std) / math.sqrt(2.0))
    t = cdf * _TWO32
    return 0xFFFFFFFF if t >= 4294967295.0 else int(t)


def models_for(spec_kwargs, n_products):
    """Per-product DemandModel list from SupplyChainEnv's demand keywords (:489-500, :566-590)."""
    by_product = spec_kwargs.get("demand_config_by_product", False)
    rng = spec_kwargs.get("demand_range", (10, 20))
    std = spec_kwargs.get("demand_std")
    peaks = spec_kwargs.get("demand_sen_peaks")
    avg = spec_kwargs.get("avg_demand_range")
    pn = spec_kwargs.get("demand_perturb_norm", False)
    if not by_product:
        minavg, maxavg = (avg[0], avg[1]) if avg else (None, None)
        return [DemandModel(rng[0], rng[1], std, peaks, minavg, maxavg, pn) for _ in range(n_products)]
    out = []
    for p in range(n_products):
        a = avg[p] if avg is not None else None
        sd = std[p] if std is not None else None
        if isinstance(sd, (list, tuple)):  # normal(mean, [x]) broadcasts like x; [None] fails there
            if len(sd) != 1 or sd[0] is None:
                raise TypeError(f"demand_std[{p}]={sd!r} is not a standard deviation")
            sd = sd[0]
        out.append(DemandModel(rng[p][0], rng[p][1], sd,
                               peaks[p] if peaks is not None else None, a[0] if a else None, a[1] if a else None,
                               pn[p] if isinstance(pn, (list, tuple)) else pn))
    return out


def fill_config(c, models, horizon, upload):
    """Per-product model fields of an scg_sc_config; `upload(ndarray) -> address` places
    the threshold (uint32) and base (float64) tables where the kernel reads them."""
    thr, base, n_thr, n_base = [], [], 0, 0
    c.demand_models = 1
    for p, m in enumerate(models):
        c.demand_kind[p], c.demand_lo_p[p], c.demand_hi_p[p] = m.kind, m.lo, m.hi
        c.demand_pert_lo[p], c.demand_pert_n[p] = m.pert_lo, m.pert_n
        if m.kind in (NORMAL, SINE_NORMAL):
            t = m.thresholds(horizon).reshape(-1)
            c.demand_off[p], n_thr = n_thr, n_thr + t.size
            thr.append(t)
        elif m.kind == SINE_UNIFORM:
            b = m.sine_base(horizon)
            c.demand_off[p], n_base = n_base, n_base + b.size
            base.append(b)
    c.demand_thr = upload(np.ascontiguousarray(np.concatenate(thr))) if thr else None
    c.demand_base = upload(np.ascontiguousarray(np.concatenate(base))) if base else None
