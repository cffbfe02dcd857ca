"""The BeerGame oracle restatements against golden vectors produced by the reference.

tests/golden/beergame_*.npz were written by oracle/gen_golden.py, which ran the real
gym_supplychain BeerGameEnv (beergame_env.py) in the build container. These tests pin
the oracle that the GPU parity tests then use at sizes the golden files do not cover.
"""
import numpy as np
import pytest

from golden_io import beergame_cases, load_beergame
from oracle.beergame import BeerGameOracle, run_batch_episode
from oracle.philox import STREAM_DEMAND, draw_words
from oracle.poisson import poisson_invert, poisson_thresholds

CASES = beergame_cases()
FIELDS = ["obs", "inventory", "backlog", "orders_placed", "reward", "inventory_costs", "backlog_costs",
          "all_orders_placed", "reset_obs"]


def test_golden_present():
    assert {"default_poisson", "vardelay_negact", "delay_collide", "levels3_fixed", "levels6_short",
            "levels1"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_batch_oracle_matches_reference(name):
    g = load_beergame(name)
    out = run_batch_episode(g["info"], g["demand"], g["actions"])
    for f in FIELDS:
        assert np.array_equal(out[f], g["ref_" + f]), f


@pytest.mark.parametrize("name", CASES)
def test_single_env_oracle_matches_reference(name):
    g = load_beergame(name)
    T, N, L = g["actions"].shape
    for n in range(min(N, 6)):
        env = BeerGameOracle(dict(g["info"], customer_demand=g["demand"][n].tolist()))
        assert np.array_equal(env.reset(), g["ref_reset_obs"][n])
        for w in range(T):
            obs, r, done, info = env.step(g["actions"][w, n].astype(np.int64))
            assert np.array_equal(obs, g["ref_obs"][w, n])
            assert r == g["ref_reward"][w, n] and done == g["ref_done"][w, n] and info == {}
            assert np.array_equal(env.incoming_orders, g["ref_incoming_orders"][w, n])
            if n < g["ref_shipments"].shape[1]:   # the whole absolute-week table (:46-52)
                assert np.array_equal(env.shipments, g["ref_shipments"][w, n])
        assert g["ref_past_horizon_raises"][n]
        with pytest.raises(IndexError):
            env.step(np.zeros(L, dtype=np.int64))


@pytest.mark.parametrize("name", [c for c in CASES if c != "levels3_fixed"])
def test_golden_demand_is_philox_poisson(name):
    """The golden demand tables are the Philox/Poisson draws the device makes."""
    g = load_beergame(name)
    thr = poisson_thresholds(float(g["lam"]))
    assert np.array_equal(thr, g["poisson_thresholds"])
    N, T = g["demand"].shape
    words = draw_words(int(g["seed"]), np.arange(N), int(g["episode"]), T, STREAM_DEMAND)
    assert np.array_equal(poisson_invert(words, thr), g["demand"])


def test_poisson_distribution():
    lam = 8.0
    thr = poisson_thresholds(lam)
    words = draw_words(99, np.arange(4096), 0, 64, STREAM_DEMAND)
    x = poisson_invert(words, thr)
    assert abs(x.mean() - lam) < 0.05 and abs(x.var() - lam) < 0.2


def test_poisson_table_edges():
    assert poisson_thresholds(0.0).tolist() == [0xFFFFFFFF]
    with pytest.raises(ValueError):
        poisson_thresholds(-1.0)
    with pytest.raises(ValueError):
        poisson_thresholds(1000.0)


# ---- BeerGameEnv2 ----------------------------------------------------------------------
from golden_io import beergame2_cases, load_beergame2  # noqa: E402
from oracle.beergame import BeerGame2Oracle  # noqa: E402


@pytest.mark.parametrize("name", beergame2_cases())
def test_beergame2_oracle_matches_reference(name):
    g = load_beergame2(name)
    T, N, L = g["actions"].shape
    kw = {k: v for k, v in g["kwargs"].items() if k not in ("customer_demand", "shipment_delays", "max_order",
                                                              "weeks", "levels")}
    for n in range(N):
        o = BeerGame2Oracle(weeks=T, levels=L, customer_demand=g["demand"][n], shipment_delays=g["delays"][n].tolist(),
                            **kw)
        assert np.array_equal(o.reset(), g["ref_reset_obs"][n])
        for w in range(T):
            obs, r, done, info = o.step(g["actions"][w, n])
            assert np.array_equal(obs, g["ref_obs"][w, n]) and r == g["ref_reward"][w, n] and isinstance(r, int)
        for k in ("inventory_costs", "backlog_costs", "penalty_costs"):
            assert np.array_equal(getattr(o, k), g["ref_" + k][n])


def test_beergame2_tables_are_philox_draws():
    import sys
    sys.path.insert(0, "oracle")
    from oracle.gen_golden_bg2 import CASES, case_tables
    for name in beergame2_cases():
        g = load_beergame2(name)
        demand, delays = case_tables(CASES[name])
        assert np.array_equal(demand, g["demand"]) and np.array_equal(delays, g["delays"])
