"""Generate tests/golden/beergame2_*.npz from the REFERENCE BeerGameEnv2 — build container only.

Each env is the reference's BeerGameEnv2 built with explicit per-env customer_demand and
shipment_delays lists (its non-stochastic constructor path, beergame2_env.py:41-55), equal
to the tables scgpu draws on device for the stochastic ranges (oracle/philox.py, streams 4
and 5: randint(low, high) per week, high exclusive, as beergame2_env.py:76-77), driven by
explicit integer actions in [0, max_order). Without /root/reference nothing is written.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REFERENCE = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
from oracle.philox import draw_words  # noqa: E402

STREAM_BG2_DEMAND, STREAM_BG2_DELAY = 4, 5

CASES = {
    # the class defaults, fixed demand list and constant delay
    "defaults": dict(kw={}, n_envs=16, seed=0, episode=0),
    # stochastic demand (0..15) and delays (0..4): per-env tables, negative penalties hit
    "stochastic": dict(kw=dict(customer_demand=(0, 16), shipment_delays=(0, 5), max_stock=20, max_order=25,
                               exceeded_capacity_penalty=7),
                       n_envs=32, seed=21, episode=2),
    # 6 levels, short horizon, per-week delay list
    "levels6": dict(kw=dict(levels=6, weeks=18, initial_inventory=[5, 9, 12, 3, 20, 8], max_stock=15,
                            customer_demand=(2, 11), shipment_delays=[1, 0, 3, 2, 2, 1] * 3, inv_cost=2,
                            backlog_cost=3, initial_shipment=6, initial_orders=5),
                    n_envs=16, seed=5, episode=0),
}


def uniform_table(seed, n, episode, T, lo, hi, stream):
    """randint(lo, hi) (hi exclusive) per week from Philox words."""
    w = draw_words(seed, np.arange(n), episode, T, stream).astype(np.uint64)
    return lo + ((w * np.uint64(hi - lo)) >> np.uint64(32)).astype(np.int64)


def case_tables(spec):
    kw = spec["kw"]
    T = kw.get("weeks", 35)
    N = spec["n_envs"]
    dem = kw.get("customer_demand", [4] * 4 + [8] * 31)
    if isinstance(dem, tuple) or (isinstance(dem, list) and len(dem) == 2):
        demand = uniform_table(spec["seed"], N, spec["episode"], T, dem[0], dem[1], STREAM_BG2_DEMAND)
    else:
        demand = np.tile(np.asarray(dem[:T], dtype=np.int64), (N, 1))
    dl = kw.get("shipment_delays", 2)
    if isinstance(dl, int):
        delays = np.full((N, T), dl, dtype=np.int64)
    elif isinstance(dl, tuple) or (isinstance(dl, list) and len(dl) == 2):
        delays = uniform_table(spec["seed"], N, spec["episode"], T, dl[0], dl[1], STREAM_BG2_DELAY)
    else:
        delays = np.tile(np.asarray(dl, dtype=np.int64), (N, 1))
    return demand, delays


def main():
    if not os.path.isdir(os.path.join(REFERENCE, "gym_supplychain")):
        print("gen_golden_bg2: /root/reference absent; keeping committed fixtures")
        return 0
    sys.path.insert(0, REFERENCE)
    sys.path.insert(0, os.path.join(HERE, "refharness"))
    from gym_supplychain.envs import BeerGameEnv2
    for name, spec in CASES.items():
        kw = dict(spec["kw"])
        T, L, N = kw.get("weeks", 35), kw.get("levels", 4), spec["n_envs"]
        max_order = kw.get("max_order", 30)
        demand, delays = case_tables(spec)
        acts = np.random.RandomState(spec["seed"] + 100).randint(0, max_order, size=(T, N, L))
        rec = {k: np.zeros((T, N, L), dtype=np.int64) for k in ("obs", "inventory", "backlog", "orders_placed")}
        rec["reward"] = np.zeros((T, N), dtype=np.int64)
        rec["reset_obs"] = np.zeros((N, L), dtype=np.int64)
        for k in ("inventory_costs", "backlog_costs", "penalty_costs"):
            rec[k] = np.zeros((N, L))
        for n in range(N):
            ekw = dict(kw, customer_demand=[int(x) for x in demand[n]], shipment_delays=[int(x) for x in delays[n]])
            env = BeerGameEnv2(**ekw)
            rec["reset_obs"][n] = env.reset()
            for w in range(T):
                obs, r, done, info = env.step(acts[w, n])
                assert isinstance(r, int) and info == {} and done == (w == T - 1)
                rec["obs"][w, n], rec["reward"][w, n] = obs, r
                rec["inventory"][w, n], rec["backlog"][w, n] = env.inventory, env.backlog
                rec["orders_placed"][w, n] = env.orders_placed
            for k in ("inventory_costs", "backlog_costs", "penalty_costs"):
                rec[k][n] = getattr(env, k)
        kwj = {k: (list(v) if isinstance(v, tuple) else v) for k, v in kw.items()}
        path = os.path.join(OUT, f"beergame2_{name}.npz")
        np.savez_compressed(path, kwargs=np.array(repr(kwj)), seed=np.uint64(spec["seed"]),
                            episode=np.uint32(spec["episode"]), demand=demand, delays=delays, actions=acts,
                            **{"ref_" + k: v for k, v in rec.items()})
        print(f"wrote {path} ({os.path.getsize(path)} B)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
