"""The reference's hand-traced SupplyChain tests, transcribed as data.

Each trace is one reference test that seeds an env, resets it and steps explicit actions,
asserting heap contents (storage order), stocks, and in some steps ledgers, rewards and
observations. Sources (gym_supplychain/envs/tests/):

    simple_det     test_supplychain_env.py:60-127      1 product, deterministic lead time 2
    simple_stoch   test_supplychain_env.py:129-205     stochastic lead times (seed-0 matrix :141-145)
    mp_simple      test_multiproduct.py:52-121          2 products, serial chain
    mp_2perstage   test_multiproduct_2perstage.py:84-218  2 products, 2 per stage, build_info

Actions are written on the reference's [0, 1] scale (the tests pass 2a - 1). Per step:
`heaps` {node: per-product list of (time, amount)} compared with ==, `stock` {node: values}
compared with np.allclose, and optionally `ledger` {key: (units, costs)} compared with ==,
`obs` (on the [0, 1] scale, compared after 2x - 1 with np.allclose) and `reward_is_cost_sum`.
`demands` is the flattened customer_demands table (or its first rows) the seed gives.
"""
import numpy as np


def simple_chain(P=1):
    """test_supplychain_env.py:11-40 (P = 1) / test_multiproduct.py:7-38 (P = 2)."""
    if P == 1:
        base = dict(initial_stock=10, stock_capacity=100, stock_cost=1)
        sup = dict(supply_capacity=50, supply_cost=5)
        fac = dict(processing_capacity=100, processing_cost=10)
        link = dict(dest_costs=[[2, 2]], ship_capacity=[100, 100])
        env = dict(num_products=1, unmet_demand_cost=1000, exceeded_stock_capacity_cost=1000,
                   exceeded_process_capacity_cost=1000, exceeded_ship_capacity_cost=1000, demand_range=(0, 5),
                   processing_ratio=2, total_time_steps=5)
    else:
        base = dict(initial_stock=[10, 20], stock_capacity=[100, 200], stock_cost=[1, 2])
        sup = dict(supply_capacity=[50, 50], supply_cost=[5, 10])
        fac = dict(processing_capacity=50, processing_cost=[10, 20])
        link = dict(dest_costs=[[2], [3]], ship_capacity=[100, 100])
        env = dict(num_products=2, unmet_demand_cost=1000, exceeded_stock_capacity_cost=101,
                   exceeded_process_capacity_cost=102, exceeded_ship_capacity_cost=103, demand_range=(0, 5),
                   processing_ratio=2, total_time_steps=5)
    nodes = {"Supplier": dict(base, **sup, destinations=["Factory"], **link),
             "Factory": dict(base, **fac, destinations=["Wholesal"], **link),
             "Wholesal": dict(base, destinations=["Retailer"], **link),
             "Retailer": dict(base, last_level=True)}
    return nodes, env


def two_per_stage_mp_chain():
    """test_multiproduct_2perstage.py:10-67: every node's parameters differ."""
    def node(stock, cap, cost, **kw):
        return dict(initial_stock=stock, stock_capacity=cap, stock_cost=cost, **kw)
    fac, whs, ret = ["Factory1", "Factory2"], ["Wholesal1", "Wholesal2"], ["Retailer1", "Retailer2"]
    nodes = {
        "Supplier1": node([11, 1], [20, 10], [1, 2], initial_supply=[[1, 4], [2, 3]], supply_capacity=[50, 60],
                          supply_cost=[10, 11], destinations=fac, dest_costs=[[1, 2], [0, 1]], ship_capacity=[100, 101]),
        "Supplier2": node([12, 2], [21, 11], [3, 4], initial_supply=[[3, 1], [4, 2]], supply_capacity=[100, 110],
                          supply_cost=[20, 21], destinations=fac, dest_costs=[[3, 4], [2, 3]], ship_capacity=[102, 103]),
        "Factory1": node([13, 3], [22, 12], [3, 4], initial_shipments=[[1, 2], [3, 4]], processing_capacity=40,
                         processing_cost=[15, 16], destinations=whs, dest_costs=[[5, 6], [4, 5]],
                         ship_capacity=[104, 105]),
        "Factory2": node([14, 4], [23, 13], [1, 2], initial_shipments=[[4, 3], [2, 1]], processing_capacity=30,
                         processing_cost=[20, 21], destinations=whs, dest_costs=[[7, 8], [6, 7]],
                         ship_capacity=[106, 107]),
        "Wholesal1": node([15, 5], [24, 14], [5, 6], initial_shipments=[[5, 6], [7, 8]], destinations=ret,
                          dest_costs=[[9, 10], [8, 9]], ship_capacity=[108, 109]),
        "Wholesal2": node([16, 6], [25, 15], [6, 5], initial_shipments=[[8, 7], [6, 5]], destinations=ret,
                          dest_costs=[[11, 12], [10, 11]], ship_capacity=[110, 111]),
        "Retailer1": node([17, 7], [26, 16], [7, 8], initial_shipments=[[0, 5], [10, 15]], last_level=True),
        "Retailer2": node([18, 8], [27, 17], [8, 7], initial_shipments=[[15, 10], [5, 0]], last_level=True),
    }
    env = dict(num_products=2, unmet_demand_cost=100, exceeded_stock_capacity_cost=101,
               exceeded_process_capacity_cost=102, exceeded_ship_capacity_cost=103, demand_range=(0, 100),
               processing_ratio=[2, 3], stochastic_leadtimes=False, avg_leadtime=2, max_leadtime=2,
               total_time_steps=5, build_info=True)
    return nodes, env


SUPPLY_1P = [1, 0, 0, 0, 0, 0]
ALL_1P = [1] * 6
EMPTY1 = [[]]


def _simple(stoch):
    if not stoch:
        steps = [
            (SUPPLY_1P, {0: [[(3, 50)]], 1: EMPTY1, 2: EMPTY1, 3: EMPTY1}, {0: [10], 1: [10], 2: [10], 3: [10 - 4]}),
            (ALL_1P, {0: [[(3, 50), (4, 50)]], 1: [[(4, 10)]], 2: [[(4, 5)]], 3: [[(4, 10)]]},
             {0: [0], 1: [0], 2: [0], 3: [max(0, 10 - 9)]}),
            (ALL_1P, {0: [[(4, 50), (5, 50)]], 1: [[(4, 10), (5, 50)]], 2: [[(4, 5)]], 3: [[(4, 10)]]},
             {0: [0], 1: [0], 2: [0], 3: [max(0, 10 - 9)]}),
            (ALL_1P, {0: [[(5, 50), (6, 50)]], 1: [[(5, 50), (6, 50)]], 2: [[(6, 5)]], 3: [[(6, 5)]]},
             {0: [0], 1: [0], 2: [0], 3: [max(0, 20 - 12)]}),
            (ALL_1P, {0: [[(6, 50), (7, 50)]], 1: [[(6, 50), (7, 50)]], 2: [[(6, 5), (7, 25)]], 3: [[(6, 5)]]},
             {0: [0], 1: [0], 2: [0], 3: [max(0, 20 - 15)]}),
        ]
        return dict(chain=simple_chain(1), env=dict(stochastic_leadtimes=False, avg_leadtime=2, max_leadtime=2),
                    seed=0, demands=[4, 5, 0, 3, 3, 3], leadtimes=None, steps=steps)
    steps = [
        (SUPPLY_1P, {0: [[(4, 50)]], 1: EMPTY1, 2: EMPTY1, 3: EMPTY1}, {0: [10], 1: [10], 2: [10], 3: [10 - 4]}),
        (ALL_1P, {0: [[(4, 50), (5, 50)]], 1: [[(4, 10)]], 2: [[(3, 5)]], 3: [[(4, 10)]]},
         {0: [0], 1: [0], 2: [0], 3: [max(0, 10 - 9)]}),
        (ALL_1P, {0: [[(4, 50), (5, 50), (5, 50)]], 1: [[(4, 10)]], 2: EMPTY1, 3: [[(4, 10), (6, 5)]]},
         {0: [0], 1: [0], 2: [0], 3: [max(0, 10 - 9)]}),
        (ALL_1P, {0: [[(5, 50), (5, 50), (6, 50)]], 1: [[(6, 50)]], 2: [[(6, 5)]], 3: [[(6, 5)]]},
         {0: [0], 1: [0], 2: [0], 3: [max(0, 20 - 12)]}),
        (ALL_1P, {0: [[(6, 50), (6, 50)]], 1: [[(6, 50), (6, 100)]], 2: [[(6, 5)]], 3: [[(6, 5)]]},
         {0: [0], 1: [0], 2: [0], 3: [max(0, 20 - 15)]}),
    ]
    return dict(chain=simple_chain(1), env=dict(stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4), seed=0,
                demands=[4, 5, 0, 3, 3, 3],
                leadtimes=[[3, 1, 1, 1], [3, 2, 1, 2], [2, 3, 2, 3], [2, 2, 2, 1], [1, 1, 1, 2]], steps=steps)


def _mp_simple():
    sup, allv = [1, 1, 0, 0, 0, 0, 0, 0], [1] * 8
    e2 = [[], []]
    z = [0.0, 0.0]
    steps = [
        (sup, {0: [[(3, 50.0)], [(3, 50.0)]], 1: e2, 2: e2, 3: e2}, {0: [10, 20], 1: [10, 20], 2: [10, 20], 3: [6, 15]}),
        (allv, {0: [[(3, 50), (4, 50)], [(3, 50), (4, 50)]], 1: [[(4, 10)], [(4, 20)]], 2: [[(4, 5)], [(4, 10)]],
                3: [[(4, 10)], [(4, 20)]]}, {0: z, 1: z, 2: z, 3: [6, 12]}),
        (allv, {0: [[(4, 50), (5, 50)], [(4, 50), (5, 50)]], 1: [[(4, 10), (5, 50)], [(4, 20), (5, 50)]],
                2: [[(4, 5)], [(4, 10)]], 3: [[(4, 10)], [(4, 20)]]}, {0: z, 1: z, 2: z, 3: [3, 9]}),
        (allv, {0: [[(5, 50), (6, 50)], [(5, 50), (6, 50)]], 1: [[(5, 50), (6, 50)], [(5, 50), (6, 50)]],
                2: [[(6, 5)], [(6, 10)]], 3: [[(6, 5)], [(6, 10)]]}, {0: z, 1: z, 2: z, 3: [12, 26]}),
        (allv, {0: [[(6, 50), (7, 50)], [(6, 50), (7, 50)]], 1: [[(6, 50), (7, 50)], [(6, 50), (7, 50)]],
                2: [[(6, 5), (7, 25)], [(6, 10)]], 3: [[(6, 5)], [(6, 10)]]}, {0: z, 1: [0.0, 50.0], 3: [7, 24]}),
    ]
    return dict(chain=simple_chain(2), env=dict(stochastic_leadtimes=False, avg_leadtime=2, max_leadtime=2), seed=0,
                demands=[4, 5, 0, 3, 3, 3, 1, 3, 5, 2, 4, 0], leadtimes=None, steps=steps)


def _mp_2perstage():
    half = 2 * [0.5, 0.5, 0.25, 0.5, 0.25, 0.5] + 4 * [0.25, 0.5, 0.25, 0.5]
    second = 2 * [1.0, 0.5, 0.5, 1.0, 0.25, 0.5] + 4 * [0.5, 1.0, 0.25, 0.5]
    # step 1: node heaps, stocks, ledger (units, costs), observation
    h1 = {0: [[(2, 4), (3, 25)], [(2, 3), (3, 30)]],
          1: [[(2, 1), (3, 50)], [(2, 2), (3, 55)]],
          2: [[(2, 2), (3, 3.75), (3, 3)], [(2, 4), (3, 1.5), (3, 0.75)]],
          3: [[(2, 3), (3, 3.75), (3, 3)], [(2, 1), (3, 1.5), (3, 0.75)]],
          4: [[(2, 6), (3, 2.25), (3, 1.75)], [(2, 8), (3, 0.5), (3, 0.5)]],
          5: [[(2, 7), (3, 2.25), (3, 1.75)], [(2, 5), (3, 0.5), (3, 0.5)]],
          6: [[(2, 5), (3, 6), (3, 5)], [(2, 15), (3, 3), (3, 3)]],
          7: [[(2, 10), (3, 6), (3, 5)], [(2, 0), (3, 3), (3, 3)]]}
    s1 = {0: [6, 1.5], 1: [7.5, 3], 2: [7, 3], 3: [9, 3], 4: [10, 6], 5: [12, 6], 6: [0, 0], 7: [0, 0]}
    unmet = [44 - (17 + 0) + 64 - (18 + 15 - 6), 47 - (7 + 10 - 1) + 67 - (8 + 5)]
    led1 = {
        "stock": ([6 + 7.5 + 7 + 9 + 10 + 12, 1.5 + 3 + 3 + 3 + 6 + 6],
                  [6 * 1 + 7.5 * 3 + 7 * 3 + 9 * 1 + 10 * 5 + 12 * 6, 1.5 * 2 + 3 * 4 + 3 * 4 + 3 * 2 + 6 * 6 + 6 * 5]),
        "stock_pen": ([6, 1], [101 * 6, 101 * 1]),
        "supply": ([25 + 50, 30 + 55], [25 * 10 + 50 * 20, 30 * 11 + 55 * 21]),
        "process": ([7 + 9, 3 + 3], [7 * 15 + 9 * 20, 3 * 16 + 3 * 21]),
        "process_pen": ([0, 0], [0, 0]),
        "ship": ([3.75 + 3 + 3.75 + 3 + 2.25 + 1.75 + 2.25 + 1.75 + 6 + 5 + 6 + 5,
                  1.5 + 0.75 + 1.5 + 0.75 + 0.5 + 0.5 + 0.5 + 0.5 + 3 + 3 + 3 + 3],
                 [3.75 * 3 + 3 * 1 + 3.75 * 4 + 3 * 2 + 2.25 * 7 + 1.75 * 5 + 2.25 * 8 + 1.75 * 6 + 6 * 11 + 5 * 9
                  + 6 * 12 + 5 * 10,
                  1.5 * 2 + 0.75 * 0 + 1.5 * 3 + 0.75 * 1 + 0.5 * 6 + 0.5 * 4 + 0.5 * 7 + 0.5 * 5 + 3 * 10 + 3 * 8
                  + 3 * 11 + 3 * 9]),
        "ship_pen": ([0, 0], [0, 0]),
        "unmet_dem": (unmet, [100 * unmet[0], 100 * unmet[1]]),
    }
    # observation after step 1: next demands, then per node stocks and in-transit bins (:762-791)
    f1, f2, w1, w2, r1, r2 = 100 + 102, 101 + 103, 104 + 106, 105 + 107, 108 + 110, 109 + 111
    obs1 = [67 / 100, 9 / 100, 83 / 100, 21 / 100,
            6 / 20, 1.5 / 10, 4 / 50, 25 / 50, 3 / 60, 30 / 60,
            7.5 / 21, 3 / 11, 1 / 100, 50 / 100, 2 / 110, 55 / 110,
            7 / 22, 3 / 12, 2 / f1, (3 + 3.75) / f1, 4 / f1, (1.5 + 0.75) / f1,
            9 / 23, 3 / 13, 3 / f2, (3 + 3.75) / f2, 1 / f2, (1.5 + 0.75) / f2,
            10 / 24, 6 / 14, 6 / w1, (2.25 + 1.75) / w1, 8 / w1, (0.5 + 0.5) / w1,
            12 / 25, 6 / 15, 7 / w2, (2.25 + 1.75) / w2, 5 / w2, (0.5 + 0.5) / w2,
            0 / 26, 0 / 16, 5 / r1, (6 + 5) / r1, 15 / r1, (3 + 3) / r1,
            0 / 27, 0 / 17, 10 / r2, (6 + 5) / r2, 0 / r2, (3 + 3) / r2,
            (5 - 1) / 5]
    fac2 = [[(3, 3), (3, 3.75), (4, (7.5 + 1) / 2), (4, (6 + 4) / 2)],
            [(3, 0.75), (3, 1.5), (4, (3 + 2) / 4), (4, (1.5 + 3) / 4)]]
    whs2 = [[(3, 1.75), (3, 2.25), (4, (9 + 3) / 2 / 2), (4, (7 + 2) / 2 / 2)],
            [(3, 0.5), (3, 0.5), (4, (3 + 1) / 3 / 4), (4, (3 + 4) / 3 / 4)]]
    ret2 = [[(3, 5), (3, 6), (4, (12 + 7) / 2), (4, (10 + 6) / 2)],
            [(3, 3), (3, 3), (4, (6 + 5) / 4), (4, (6 + 8) / 4)]]
    h2 = {0: [[(3, 25), (4, 50)], [(3, 30), (4, 30)]], 1: [[(3, 50), (4, 100)], [(3, 55), (4, 55)]],
          2: fac2, 3: fac2, 4: whs2, 5: whs2, 6: ret2, 7: ret2}
    s2 = {0: [0, (1.5 + 3) / 2], 1: [0, (3 + 2) / 2], 2: [0, (3 + 4) / 2], 3: [0, (3 + 1) / 2], 4: [0, (6 + 8) / 2],
          5: [0, (6 + 5) / 2], 6: [0, 0 + 15 - 9], 7: [0, 0]}
    steps = [(half, h1, s1, dict(ledger=led1, obs=obs1, reward_is_cost_sum=True)), (second, h2, s2)]
    return dict(chain=two_per_stage_mp_chain(), env={}, seed=0, demands=[44, 47, 64, 67, 67, 9, 83, 21],
                demand_rows=2, leadtimes=None, steps=steps)


TRACES = {"simple_det": _simple(False), "simple_stoch": _simple(True), "mp_simple": _mp_simple(),
          "mp_2perstage": _mp_2perstage()}


def run_trace(trace, make_env):
    """Replay a trace on an env from make_env(nodes_info, **env_kwargs) with the reference's
    attribute surface (seed/reset/step, customer_demands, leadtimes, nodes[i].stock and
    .shipments_by_prod). Raises AssertionError on the first difference."""
    nodes, env_kw = trace["chain"]
    env = make_env(nodes, **dict(env_kw, **trace["env"]))
    env.seed(trace["seed"])
    env.reset()
    rows = trace.get("demand_rows")
    dem = np.asarray(env.customer_demands)
    dem = dem[:rows] if rows else dem
    assert dem.flatten().tolist() == trace["demands"]
    if trace["leadtimes"] is not None:
        assert np.asarray(env.leadtimes).tolist() == trace["leadtimes"]
    if rows is None:  # the serial chains start with nothing in transit
        for node in env.nodes:
            assert node.shipments_by_prod == [[] for _ in range(env.num_products)]
    for t, step in enumerate(trace["steps"], start=1):
        action, heaps, stocks = step[:3]
        extra = step[3] if len(step) > 3 else {}
        obs, reward, _, info = env.step(2 * np.array(action) - 1)
        for i, want in heaps.items():
            assert env.nodes[i].shipments_by_prod == want, (t, i, env.nodes[i].shipments_by_prod, want)
        for i, want in stocks.items():
            assert np.allclose(env.nodes[i].stock, want), (t, i, env.nodes[i].stock, want)
        if "ledger" in extra:
            units, costs = info["sc_episode"]["units"], info["sc_episode"]["costs"]
            for key, (u, c) in extra["ledger"].items():
                assert list(units[key]) == u and list(costs[key]) == c, (t, key, units[key], costs[key], u, c)
            if extra.get("reward_is_cost_sum"):
                assert reward == -sum(sum(costs[k]) for k in costs)
        if "obs" in extra:
            assert np.allclose(obs, 2 * np.array(extra["obs"]) - 1), t
    return env
