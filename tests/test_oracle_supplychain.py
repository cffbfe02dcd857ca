"""SupplyChain oracle and configuration against the reference.

* tests/golden/sc_*.npz come from the reference SupplyChainEnv family (oracle/gen_golden_sc.py):
  the oracle must reproduce observations, rewards, stocks and every in-transit heap in
  storage order exactly.
* The scenario builders must produce the nodes_info dicts captured from the reference.
* The reference's own hand-traced known answers (test_supplychain_2perstage_env.py
  test_chain_dynamics: reset/step observations and rewards for explicit actions, with the
  RandomState(0) demand table) replayed on the oracle.
"""
import json

import numpy as np
import pytest

from golden_io import load_sc, sc_cases
from oracle.supplychain import SupplyChainOracle

CASES = sc_cases()


def test_golden_present():
    assert {"2perstage", "2perstage_full", "2perstage_stoch", "2perstage_edges", "ntom", "nperstage_3p_stoch",
            "multiproduct", "seasonal", "byproduct", "byproduct_normal"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    g = load_sc(name)
    meta = g["meta"]
    T, N = meta["T"], g["obs"].shape[1]
    for n in range(N):
        o = SupplyChainOracle(meta["nodes_info"], **g["oracle_kwargs"])
        obs = o.reset(g["demands"][n], g["leadtimes"][n] if meta["n_lt"] else None)
        assert np.array_equal(obs, g["obs"][0, n])
        for t in range(T):
            obs, r, done, info = o.step(g["actions"][t, n].copy())
            assert np.array_equal(obs, g["obs"][t + 1, n]), (name, n, t)
            assert r == g["reward"][t, n], (name, n, t)
            assert done == (t == T - 1) and info == {}
            stock = np.array([np.asarray(nd.stock, dtype=np.float64) for nd in o.nodes])
            assert np.array_equal(stock, g["stock"][t + 1, n])
            for i, heaps in enumerate(o.heaps()):
                for p, h in enumerate(heaps):
                    size = int((g["heap_t"][t + 1, n, i, p] >= 0).sum())
                    assert [x[0] for x in h] == g["heap_t"][t + 1, n, i, p, :size].tolist()
                    assert [float(x[1]) for x in h] == g["heap_v"][t + 1, n, i, p, :size].tolist()


@pytest.mark.parametrize("name", CASES)
def test_scenario_builders_match_reference(name):
    from gym_supplychain_amd.envs import scenarios
    g = load_sc(name)
    meta = g["meta"]
    builder = {"SupplyChain2perStageEnv": scenarios.two_per_stage_nodes,
               "SupplyChainNPerStage": scenarios.n_per_stage_nodes,
               "SupplyChainMultiProduct": scenarios.multi_product_nodes,
               "SupplyChain2perStageSeasonalEnv": scenarios.two_per_stage_seasonal_nodes,
               "SupplyChainMultiProduct_DemConfigByProd":
                   lambda **kw: scenarios.multi_product_nodes(**scenarios.by_product_demand_kwargs(**kw)),
               }[meta["factory"]]
    nodes, kw = builder(**meta["factory_kwargs"])
    assert json.loads(json.dumps(nodes)) == meta["nodes_info"]
    ref_kw = json.loads(json.dumps(meta["kwargs"]))
    assert json.loads(json.dumps(kw)) == ref_kw


def test_spec_sizes_match_reference():
    from gym_supplychain_amd.envs import SupplyChainSpec
    for name in CASES:
        g = load_sc(name)
        meta = g["meta"]
        spec = SupplyChainSpec(meta["nodes_info"], **meta["kwargs"])
        assert (spec.n_actions, spec.n_obs) == (meta["n_act"], meta["n_obs"])
        if meta["n_lt"]:
            assert spec.n_leadtimes == meta["n_lt"]


# Known answers of the reference's own test (test_supplychain_2perstage_env.py:28-170):
# SupplyChain2perStageEnv(total_time_steps=5, ship_capacity=250), seed 0. Data only.
KA_DEMANDS = [15, 10, 13, 13, 17, 19, 13, 15, 12, 14, 17, 16]
KA_RESET_OBS = [0., -1., -1., 0., 0., -1., -0.2, -0.2, -1., -0.76, -0.76, -1., -0.76, -0.76, -1., -0.92, -0.92, -1.,
                -0.92, -0.92, -1., -0.92, -0.92, -1., -0.92, -0.92, 1.]
KA_ACTIONS = [[1] + [0] * 13, [0, 1, 1] * 2 + [1] * 8] + [[0, 0.5, 1] * 2 + [0.5, 1] * 4] * 3
KA_OBS = [
    [-0.4, -0.4, -0.4, 0., 1., -0.6, -0.2, -1., -0.4, -0.76, -1., -0.6, -0.76, -1., -0.8, -0.92, -1., -0.86666667,
     -0.92, -1., -0.95, -0.92, -1., -0.93333333, -0.92, -1., 0.6],
    [0.4, 0.8, -1., 1., -1., -1., -1., -1., -1., -1., -0.04, -1., -1., -1., -1., -1., -0.68, -1., -1., -1., -0.88, -1.,
     -0.68, -0.88666667, -1., -1., 0.2],
    [-0.4, 0., -1., -1., -1., -1., -1., -1., -1., -0.04, -0.76, -1., -1., -0.76, -1., -0.68, -1., -1., -1., -1., -1.,
     -0.68, -1., -1., -1., -1., -0.2],
    [-0.6, -0.2, -1., -1., -1., -1., -1., -1., -1., -0.76, -1., -1., -0.76, -1., -1., -1., -0.86666667, -1., -1.,
     -0.86666667, -0.33, -1., -0.84, -1., -1., -0.84, -0.6],
    [0.4, 0.2, -1., -1., -1., -1., -1., -1., -1., -1., -1., -1., -1., -1., -1., -0.86666667, -0.92, -1., -0.86666667,
     -0.92, -0.45, -0.84, -1., -1., -0.84, -1., -1.],
]
KA_REWARDS = [-1015.0, -3469.0, -1752.0, -6400.333, -4479.0]


def test_reference_known_answers_chain_dynamics():
    from gym_supplychain_amd.envs.scenarios import two_per_stage_nodes
    nodes, kw = two_per_stage_nodes(total_time_steps=5, ship_capacity=250)
    o = SupplyChainOracle(nodes, **{k: kw[k] for k in kw if k in
                                    ("num_products", "unmet_demand_cost", "exceeded_stock_capacity_cost",
                                     "exceeded_process_capacity_cost", "exceeded_ship_capacity_cost", "demand_range",
                                     "processing_ratio", "stochastic_leadtimes", "avg_leadtime", "max_leadtime",
                                     "total_time_steps")})
    # the reference's seed(0) table: RandomState(0).randint(10, 21, (T+1, R, P)) (demands_generator.py:33-36)
    dem = np.random.RandomState(0).randint(10, 21, size=(6, 2, 1))
    assert dem.flatten().tolist() == KA_DEMANDS
    assert np.allclose(o.reset(dem), KA_RESET_OBS)
    for act, want_obs, want_r in zip(KA_ACTIONS, KA_OBS, KA_REWARDS):
        obs, r, _, _ = o.step(2 * np.array(act) - 1)
        assert np.allclose(obs, want_obs)
        assert np.round(r, 3) == want_r


KIND = {int: 0, float: 1, np.float32: 2, np.float64: 3, np.int64: 4}


@pytest.mark.parametrize("name", CASES)
def test_oracle_ledgers_match_reference(name):
    """build_info=True: info['sc_episode'] (:684-695, :750-760) — every cost/unit entry's value
    and NumPy type after every step, as the reference recorded them."""
    from oracle.supplychain import LEDGER_KEYS
    g = load_sc(name)
    meta = g["meta"]
    T, N = meta["T"], g["obs"].shape[1]
    for n in range(N):
        o = SupplyChainOracle(meta["nodes_info"], build_info=True, **g["oracle_kwargs"])
        o.reset(g["demands"][n], g["leadtimes"][n] if meta["n_lt"] else None)
        for t in range(T):
            _, r, _, info = o.step(g["actions"][t, n].copy())
            led = info["sc_episode"]
            assert float(led["rewards"]) == g["led_rewards"][t, n]
            for j, key in enumerate(LEDGER_KEYS):
                for part, f in (("costs", "led_cost"), ("units", "led_units")):
                    got = led[part][key]
                    assert [float(x) for x in got] == g[f][t, n, j].tolist(), (name, n, t, key, part)
                    assert [KIND[type(x)] for x in got] == g[f + "_k"][t, n, j].tolist(), (name, n, t, key, part)


# Known answers of the reference's ledger tests (test_multiproduct.py:123-237): a 4-node
# serial chain with 2 products, penalties 101/102/103, RandomState(0) demand in [0, 5].
# Data only: (actions per step, then {key: (units, costs)} asserted after the last step).
def ka_multiproduct_chain():
    nodes = {}
    common = dict(initial_stock=[10, 20], stock_capacity=[100, 200], stock_cost=[1, 2])
    nodes["Supplier"] = dict(common, supply_capacity=[50, 50], supply_cost=[5, 10], destinations=["Factory"],
                             dest_costs=[[2], [3]], ship_capacity=[100, 100])
    nodes["Factory"] = dict(common, processing_capacity=50, processing_cost=[10, 20], destinations=["Wholesal"],
                            dest_costs=[[2], [3]], ship_capacity=[100, 100])
    nodes["Wholesal"] = dict(common, destinations=["Retailer"], dest_costs=[[2], [3]], ship_capacity=[100, 100])
    nodes["Retailer"] = dict(common, last_level=True)
    kw = dict(num_products=2, unmet_demand_cost=1000, exceeded_stock_capacity_cost=101,
              exceeded_process_capacity_cost=102, exceeded_ship_capacity_cost=103, demand_range=(0, 5),
              processing_ratio=2, stochastic_leadtimes=False, avg_leadtime=2, max_leadtime=2)
    return nodes, kw


KA_SUPPLY = [1, 1, 0, 0, 0, 0, 0, 0]
KA_SEND_ALL = [1] * 8
KA_SUPPLIER_FULL = [1, 1, 1, 1, 0, 0, 0, 0]
KA_LEDGERS = {
    "basic": (5, [KA_SUPPLY, KA_SEND_ALL, KA_SEND_ALL, KA_SEND_ALL],
              {"stock": ([57, 122], [57, 244]), "stock_pen": ([0, 0], [0, 0]), "supply": ([200, 200], [1000, 2000]),
               "process": ([20, 40], [200, 800]), "process_pen": ([0, 0], [0, 0]), "ship": ([135, 170], [270, 510]),
               "ship_pen": ([0, 0], [0, 0]), "unmet_dem": ([0, 0], [0, 0])}),
    "pen_4": (5, [KA_SUPPLY] * 4, {"stock_pen": ([10, 0], [1010, 0])}),
    "pen_5": (5, [KA_SUPPLY] * 4 + [KA_SEND_ALL],
              {"ship_pen": ([0, 70], [0, 103 * 70]), "unmet_dem": ([3, 0], [3000, 0])}),
    "processpen": (6, [KA_SUPPLY] + [KA_SUPPLIER_FULL] * 4 + [KA_SEND_ALL],
                   {"process_pen": ([50, 140], [102 * 50, 102 * 140])}),
}


@pytest.mark.parametrize("case", sorted(KA_LEDGERS))
def test_reference_known_answers_ledgers(case):
    T, acts, want = KA_LEDGERS[case]
    nodes, kw = ka_multiproduct_chain()
    o = SupplyChainOracle(nodes, build_info=True, total_time_steps=T, **kw)
    o.reset(np.random.RandomState(0).randint(0, 6, size=(T + 1, 1, 2)))   # env.seed(0) demand table
    for a in acts:
        _, _, _, info = o.step(2 * np.array(a) - 1)
    for key, (units, costs) in want.items():
        assert info["sc_episode"]["units"][key] == units, key
        assert info["sc_episode"]["costs"][key] == costs, key
