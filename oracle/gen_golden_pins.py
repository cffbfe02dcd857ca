"""Generate tests/golden/ref_pins.npz and tests/golden/ref_tables.npz — build container only.

ref_pins.npz: the reference's episode-reward pin tests re-run with the REAL reference
(gym_supplychain imported read-only from /root/reference, gym stood in by
oracle/refharness/, whose Box.seed/sample restate gym 0.21 — SURVEY F8). Each case is a
reference test that seeds the env, resets and steps one episode with
`env.action_space.sample()`:

    test_Nperstage.py:23-53                  7 cases, env.seed(0)
    test_multiproduct_2perstage.py:221-309  11 cases (+ IncreasingCosts), env.seed(0)
    tests/utils.py:13-22 check_build_info    5 cases, env.seed(1) (test_supplychain_env.py:287-293,
                                             test_supplychain_2perstage_env.py, Seasonal :338-342)

Per case: the pinned episode reward written in the reference test (NaN where the test pins
none), and from this run the per-step rewards, the first two sampled actions, the SHA-256 of
every sampled action and of every episode table, and the final info['sc_episode'] ledger
(build_info cases). numpy 2.2 gives rewards within the tests' np.allclose of the pins but
not bit-equal to them (they predate NEP 50), so the per-step rewards of this run are the
exact target.

ref_tables.npz: the reference's own RandomState fixtures (tests/data/*.npy, loaded at
test_supplychain_env.py:227,245,276 and test_supplychain_2perstage_env.py:179,197,228,278,
296,327), stored losslessly as small integer arrays (np.load(allow_pickle=False); every
value is an integer, checked) plus the SHA-256 of each original file's array bytes.

    python oracle/gen_golden_pins.py
Nothing is written under /root/reference (tests run from the same read-only tree; the
reference test that writes a fixture is not run). Without /root/reference it exits.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REFERENCE = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.dont_write_bytecode = True

NAN = float("nan")
# (name, reference factory class, kwargs, seed, pinned reward in the reference test file)
PIN_CASES = [
    ("3perstage", "SupplyChainNPerStage", dict(nodes_per_echelon=3), 0, -60038768.011493534),
    ("3perstage_seasonal", "SupplyChainNPerStage",
     dict(nodes_per_echelon=3, demand_std=60, demand_sen_peaks=4, avg_demand_range=(100, 300),
          demand_perturb_norm=True), 0, -57730855.89812181),
    ("3perstage_3products", "SupplyChainNPerStage", dict(nodes_per_echelon=3, num_products=3), 0, -88943757.80027954),
    ("10perstage", "SupplyChainNPerStage", dict(nodes_per_echelon=10), 0, -197097090.01279718),
    ("chain_3_2_3_5", "SupplyChainNPerStage", dict(nodes_per_echelon=[3, 2, 3, 5]), 0, -120404116.66453858),
    ("chain_5_4_7_10", "SupplyChainNPerStage", dict(nodes_per_echelon=[5, 4, 7, 10]), 0, -251255147.76827675),
    ("chain_5_4_7_10_4products", "SupplyChainNPerStage", dict(nodes_per_echelon=[5, 4, 7, 10], num_products=4), 0,
     -501101931.2484466),
    ("mp", "SupplyChainMultiProduct", dict(), 0, -34704704.078214735),
    ("mp_N20", "SupplyChainMultiProduct",
     dict(demand_range=(0, 400), avg_demand_range=[100, 300], demand_std=20, demand_sen_peaks=4,
          demand_perturb_norm=True, stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4), 0, -33914245.32990393),
    ("mp_rN50", "SupplyChainMultiProduct",
     dict(demand_range=(0, 400), avg_demand_range=[100, 300], demand_std=50, demand_perturb_norm=True,
          stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4), 0, -33511405.156877503),
    ("mp_3products", "SupplyChainMultiProduct", dict(num_products=3), 0, -52509572.65837007),
    ("m3p_N20", "SupplyChainMultiProduct",
     dict(num_products=3, demand_range=(0, 400), avg_demand_range=[100, 300], demand_std=20, demand_sen_peaks=4,
          demand_perturb_norm=True, stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4), 0, -51585258.57599297),
    ("m3p_rN50", "SupplyChainMultiProduct",
     dict(num_products=3, demand_range=(0, 400), avg_demand_range=[100, 300], demand_std=50, demand_perturb_norm=True,
          stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4), 0, -51132357.668103226),
    ("mp_10products", "SupplyChainMultiProduct", dict(num_products=10), 0, -173415102.8513805),
    ("mp_build_info", "SupplyChainMultiProduct", dict(build_info=True), 0, -34704704.078214735),
    ("mp_inccosts_build_info", "SupplyChainMultiProduct_IncreasingCosts", dict(build_info=True), 0, NAN),
    ("dem_by_prod", "SupplyChainMultiProduct_DemConfigByProd",
     dict(demand_std=20, demand_perturb_norm=True, build_info=True), 0, -26065306.020432994),
    ("dem_by_prod_3p", "SupplyChainMultiProduct_DemConfigByProd",
     dict(num_products=3, demand_std=20, demand_perturb_norm=True, build_info=True), 0, -43549397.38202231),
    ("dem_by_prod_inccosts", "SupplyChainMultiProduct_DemConfigByProd_IncCosts",
     dict(demand_std=20, demand_perturb_norm=True, build_info=True), 0, -31556408.636398595),
    ("dem_by_prod_inccosts_3p", "SupplyChainMultiProduct_DemConfigByProd_IncCosts",
     dict(num_products=3, demand_std=20, demand_perturb_norm=True, build_info=True), 0, -59867745.134582885),
    # check_build_info (tests/utils.py:13-22): seed 1, Σrewards == info rewards == -Σcosts each step
    ("simple_build_info", "simple_chain", dict(stochastic_leadtimes=False, avg_leadtime=2, max_leadtime=2), 1, NAN),
    ("simple_stoch_build_info", "simple_chain", dict(stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4), 1,
     NAN),
    ("2perstage_seasonal_build_info", "SupplyChain2perStageSeasonalEnv",
     dict(stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4, demand_perturb_norm=True, build_info=True), 1,
     NAN),
]


def simple_chain_nodes():
    """test_supplychain_env.py:11-40 _create_env's chain (the values its tests pass)."""
    caps = dict(initial_stock=10, stock_capacity=100, stock_cost=1)
    nodes = {"Supplier": dict(caps, supply_capacity=50, supply_cost=5, destinations=["Factory"],
                              dest_costs=[[2, 2]], ship_capacity=[100, 100]),
             "Factory": dict(caps, processing_capacity=100, processing_cost=10, destinations=["Wholesal"],
                             dest_costs=[[2, 2]], ship_capacity=[100, 100]),
             "Wholesal": dict(caps, destinations=["Retailer"], dest_costs=[[2, 2]], ship_capacity=[100, 100]),
             "Retailer": dict(caps, last_level=True)}
    env_kw = dict(num_products=1, unmet_demand_cost=1000, exceeded_stock_capacity_cost=1000,
                  exceeded_process_capacity_cost=1000, exceeded_ship_capacity_cost=1000, demand_range=(0, 5),
                  processing_ratio=2, total_time_steps=5, build_info=True)
    return nodes, env_kw


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run_pins():
    import gym_supplychain.envs as E  # noqa: E402  (reference, read-only)
    arrays, meta = {}, {}
    for name, factory, kw, seed, pin in PIN_CASES:
        if factory == "simple_chain":
            nodes, ekw = simple_chain_nodes()
            env = E.SupplyChainEnv(nodes, **ekw, **kw)
        else:
            env = getattr(E, factory)(**kw)
        env.seed(seed)
        env.reset()
        tables = [np.asarray(env.customer_demands)]
        if getattr(env, "stochastic_leadtimes", False):
            tables.append(env.leadtimes)
        acts_hash = hashlib.sha256()
        rewards, first, done, info = [], [], False, {}
        while not done:
            a = env.action_space.sample()
            if len(first) < 2:
                first.append(a.copy())
            acts_hash.update(np.ascontiguousarray(a).tobytes())
            _, r, done, info = env.step(a)
            rewards.append(float(r))
        arrays[f"{name}/rewards"] = np.asarray(rewards, dtype=np.float64)
        arrays[f"{name}/first_actions"] = np.stack(first).astype(np.float32)
        m = dict(factory=factory, kwargs=kw, seed=seed, pin=pin, actions_sha256=acts_hash.hexdigest(),
                 tables_sha256=[_sha(t.astype(np.int64)) for t in tables], episode_reward=float(sum(rewards)),
                 n_actions=int(env.action_space.shape[0]))
        if "sc_episode" in info:
            led = info["sc_episode"]
            m["ledger"] = {part: {k: [float(x) for x in v] for k, v in led[part].items()} for part in ("costs", "units")}
            m["ledger_rewards"] = float(led["rewards"])
        meta[name] = m
        print(f"{name}: {m['episode_reward']!r} (pin {pin!r})", flush=True)
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "ref_pins.npz"), **arrays)


TABLE_FILES = ["demands_2perstage", "demands_2perstage_stocleadtimes", "demands_2perstageSeasonal",
               "demands_2perstageSeasonal_stocleadtimes", "demands_simple_chain",
               "demands_simple_chain_stocleadtimes", "leadtimes_2perstage", "leadtimes_2perstageSeasonal",
               "leadtimes_simple_chain"]


def convert_tables():
    data = os.path.join(REFERENCE, "gym_supplychain", "envs", "tests", "data")
    arrays, meta = {}, {}
    for name in TABLE_FILES:
        a = np.load(os.path.join(data, name + ".npy"), allow_pickle=False)
        assert np.array_equal(a, np.rint(a)), name
        small = a.astype(np.int16)
        assert np.array_equal(small.astype(a.dtype), a), name
        arrays[name] = small
        meta[name] = dict(dtype=str(a.dtype), shape=list(a.shape), sha256=_sha(a))
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "ref_tables.npz"), **arrays)
    print("ref_tables.npz:", {k: v["shape"] for k, v in meta.items()})


def main():
    if not os.path.isdir(REFERENCE):
        print(f"{REFERENCE} absent: keeping the committed fixtures")
        return
    sys.path.insert(0, REFERENCE)
    sys.path.insert(0, os.path.join(HERE, "refharness"))
    convert_tables()
    run_pins()


if __name__ == "__main__":
    main()
