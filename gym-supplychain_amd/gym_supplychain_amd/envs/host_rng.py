"""Host RandomState episode draws of SupplyChainEnv.reset (supplychain_env.py:630-672).

The reference draws a whole episode's customer-demand table and (stochastic lead times)
lead-time table at reset() from the env's `np.random.RandomState(seed)` (:564, :811-812):

    demand      generate_demand(rng, (T+1, R, P), ...)              :644-649
                or, demand_config_by_product, one (T+1, R) table per product   :653-661
    lead times  clip(1 + rng.poisson(avg_leadtime - 1, (T, n_lt)), 1, max_leadtime)  :670-672

`HostEpisodeDraws` makes exactly those RandomState calls, in that order, with the same
arguments (generate_demand and its three generators, demands_generator.py:3-89, restated
below), so a seeded drop-in env replays the reference's episodes draw for draw — the
reference's .npy fixtures (tests/data/) and its episode-reward pins included. The tables
go to the device once per episode and the kernels read them instead of their Philox
draws (scg_sc_config.demand_table / leadtime_table). This is reset-time randomness, as in
the reference; the step dynamics stay on the GPU.
"""
import numpy as np


def uniform_data(rng, shape, minv, maxv):
    """demands_generator.py:33-36."""
    return rng.randint(low=minv, high=maxv + 1, size=shape)


def normal_data(rng, shape, minv, maxv, std):
    """demands_generator.py:38-49: normal around the range centre, clipped, rounded."""
    data = rng.normal((maxv + minv) / 2, std, size=shape)
    np.clip(data, minv, maxv, out=data)
    return np.rint(data).astype(int)


def senoidal_data(rng, horizon, shape, minv, maxv, std, num_peaks, minavg, maxavg, perturb_norm):
    """demands_generator.py:51-89: sinusoid between minavg and maxavg plus a normal
    (or uniform in [-3 std, 3 std]) perturbation, clipped and rounded. The base is
    evaluated one period at a time with the reference's expression and operand order."""
    half_curve = (maxavg - minavg) / 2
    sin_arg = num_peaks * 2 * np.pi / horizon
    if perturb_norm:
        perturb = rng.normal(0, std, size=shape)
    else:
        perturb = rng.randint(low=-3 * std, high=3 * std + 1, size=shape)
    data = np.zeros(shape)
    for period in range(shape[0]):
        base = minavg + half_curve * (1 + np.sin(sin_arg * period))
        for d in range(shape[1]):
            data[period, d] = np.clip(base + perturb[period, d], minv, maxv)
    return np.rint(data).astype(int)


def generate_demand(rng, shape, horizon, minv, maxv, std=None, sen_peaks=None, minavg=None, maxavg=None,
                    perturb_norm=True):
    """demands_generator.py:3-31: uniform, normal or sinusoidal by the arguments given."""
    if sen_peaks is None:
        if std is None:
            return uniform_data(rng, shape, minv, maxv)
        return normal_data(rng, shape, minv, maxv, std)
    std = 0 if std is None else std
    return senoidal_data(rng, horizon, shape, minv, maxv, std, sen_peaks, minavg, maxavg, perturb_norm)


class HostEpisodeDraws:
    """SupplyChainEnv's reset-time RandomState stream for one env (:564, :644-672).

    draw() -> (customer_demands as the reference holds it, demand table int32 [T+1, R, P],
    lead times int64 [T, n_lt] or None). seed(s) restarts the stream like env.seed (:812).
    """

    def __init__(self, demand_kwargs, n_retailers, n_products, total_time_steps, n_leadtimes, stochastic_leadtimes,
                 avg_leadtime, max_leadtime, seed=None):
        kw = dict(demand_kwargs)
        self.by_product = bool(kw.get("demand_config_by_product", False))
        self.demand_range = kw.get("demand_range", (10, 20))
        self.std = kw.get("demand_std")
        self.peaks = kw.get("demand_sen_peaks")
        avg = kw.get("avg_demand_range")
        self.perturb_norm = kw.get("demand_perturb_norm", False)
        P = n_products
        if not self.by_product:                                                      # :575-579
            self.minavg, self.maxavg = (avg[0], avg[1]) if avg else (None, None)
        else:                                                                        # :580-587
            self.minavg, self.maxavg = [None] * P, [None] * P
            for p in range(P):
                if avg[p]:
                    self.minavg[p], self.maxavg[p] = avg[p][0], avg[p][1]
        self.R, self.P, self.T = n_retailers, P, total_time_steps
        self.n_lt, self.stochastic = n_leadtimes, bool(stochastic_leadtimes)
        self.avg_lt, self.max_lt = avg_leadtime, max_leadtime
        self.seed(seed)

    def seed(self, seed=None):
        self.rng = np.random.RandomState(seed)

    def draw(self):
        T, R, P = self.T, self.R, self.P
        if not self.by_product:                                                      # :641-649
            dem = generate_demand(self.rng, (T + 1, R, P), T, self.demand_range[0], self.demand_range[1],
                                  std=self.std, sen_peaks=self.peaks, minavg=self.minavg, maxavg=self.maxavg,
                                  perturb_norm=self.perturb_norm)
            table = np.asarray(dem).reshape(T + 1, R, P)
        else:                                                                        # :650-661
            dem = [generate_demand(self.rng, (T + 1, R), T, self.demand_range[p][0], self.demand_range[p][1],
                                   std=self.std[p], sen_peaks=self.peaks[p], minavg=self.minavg[p],
                                   maxavg=self.maxavg[p], perturb_norm=self.perturb_norm[p]) for p in range(P)]
            table = np.stack([np.asarray(d).reshape(T + 1, R) for d in dem], axis=-1)
        if table.size and (table.min() < -2 ** 31 or table.max() >= 2 ** 31):
            raise ValueError("customer demand does not fit int32")
        lts = None
        if self.stochastic:                                                          # :664-672
            lts = 1 + self.rng.poisson(lam=self.avg_lt - 1, size=(T, self.n_lt))
            lts = np.clip(lts, 1, self.max_lt)
        return dem, table.astype(np.int32), lts
