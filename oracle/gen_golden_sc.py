"""Generate tests/golden/sc_*.npz from the REFERENCE SupplyChainEnv — build container only.

Runs gym_supplychain's SupplyChainEnv family (imported read-only from /root/reference with
the inert gym stand-in of oracle/refharness/) per env, with explicit float32 actions and
with the episode's demand / lead-time tables replaced right after reset() by the tables
the device draws (oracle/sc_draws.py), and records per step: observation, reward, node
stocks, every in-transit heap in storage order (time, amount, amount type) and, with
build_info switched on, the episode ledgers of info['sc_episode'] (value and type of every
cost/unit entry). The
scenario's nodes_info and constructor kwargs are captured from the reference's own
factory classes and stored as JSON next to the arrays. Nothing is written under
/root/reference; without it the script exits leaving the committed fixtures alone.

    python oracle/gen_golden_sc.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REFERENCE = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

from oracle.sc_draws import sc_demand_table, sc_demand_table_models, sc_leadtime_table  # noqa: E402

# Amount type codes in recorded heaps (amounts are float32, float64 or int)
KIND = {int: 0, float: 1, np.float32: 2, np.float64: 3, np.int64: 4}
# info['sc_episode'] cost/unit categories in the reference's dict order (:416-417, :685-686)
LEDGER_KEYS = ("stock", "stock_pen", "supply", "process", "process_pen", "ship", "ship_pen", "unmet_dem")

CASES = {
    # BASELINE config 3 scenario (sc-2perstage-v0 defaults), shortened horizon
    "2perstage": dict(factory="SupplyChain2perStageEnv", kwargs=dict(total_time_steps=48), n_envs=6,
                      act="uniform", seed=11),
    # full 360-step episode of the defaults
    "2perstage_full": dict(factory="SupplyChain2perStageEnv", kwargs=dict(), n_envs=2, act="uniform", seed=12),
    # stochastic Poisson lead times (cursor quirk, :252-254), tight ship capacity -> penalties
    "2perstage_stoch": dict(factory="SupplyChain2perStageEnv",
                            kwargs=dict(total_time_steps=40, stochastic_leadtimes=True, avg_leadtime=2,
                                        max_leadtime=4, ship_capacity=90),
                            n_envs=6, act="uniform", seed=13),
    # actions outside [-1, 1] and exact grid values (ties in the sorted cut, clamps)
    "2perstage_edges": dict(factory="SupplyChain2perStageEnv",
                            kwargs=dict(total_time_steps=30, processing_capacities=[40, 35], ship_capacity=70,
                                        stock_capacities=[90, 120] * 4),
                            n_envs=6, act="edges", seed=14),
    # BASELINE config 4 scenario (ntom = SupplyChainNPerStage([8,8,8,16]), 2 products)
    "ntom": dict(factory="SupplyChainNPerStage", kwargs=dict(nodes_per_echelon=[8, 8, 8, 16], total_time_steps=12),
                 n_envs=2, act="uniform", seed=15),
    # small N-per-stage, 3 products, stochastic lead times
    "nperstage_3p_stoch": dict(factory="SupplyChainNPerStage",
                               kwargs=dict(nodes_per_echelon=[2, 3, 2, 3], num_products=3, total_time_steps=25,
                                           stochastic_leadtimes=True, avg_leadtime=3, max_leadtime=5),
                               n_envs=4, act="uniform", seed=16),
    # multi-product 2-per-stage factory (config only in the reference)
    "multiproduct": dict(factory="SupplyChainMultiProduct", kwargs=dict(total_time_steps=30), n_envs=4,
                         act="uniform", seed=17),
    # sc-2perstage-seasonal-v0: sinusoidal demand with normal perturbation (demands_generator.py:51-89)
    "seasonal": dict(factory="SupplyChain2perStageSeasonalEnv", kwargs=dict(total_time_steps=40), n_envs=4,
                     act="uniform", seed=18),
    # sc-2perstage-multiproduct-v1: demand configured per product (sinusoid, uniform and a
    # second sinusoid, uniform perturbation; per-product observation normalisation)
    "byproduct": dict(factory="SupplyChainMultiProduct_DemConfigByProd",
                      kwargs=dict(num_products=3, demand_std=6, total_time_steps=30), n_envs=4, act="uniform",
                      seed=19),
    # the same with normal perturbations and normal (non-sinusoidal) product 2
    "byproduct_normal": dict(factory="SupplyChainMultiProduct_DemConfigByProd",
                             kwargs=dict(num_products=2, demand_std=25.0, demand_perturb_norm=True,
                                         total_time_steps=30), n_envs=4, act="uniform", seed=20),
}


def demand_models(env):
    """Per-product generator settings of a reference env (:566-590), oracle/sc_draws form."""
    P = env.num_products
    if not env.demand_config_by_product:
        m = dict(lo=env.demand_range[0], hi=env.demand_range[1], std=env.demand_std, sen_peaks=env.demand_sen_peaks,
                 minavg=env.minavg_demand, maxavg=env.maxavg_demand, perturb_norm=env.demand_perturb_norm)
        return [m] * P
    return [dict(lo=env.demand_range[p][0], hi=env.demand_range[p][1], std=env.demand_std[p],
                 sen_peaks=env.demand_sen_peaks[p], minavg=env.minavg_demand[p], maxavg=env.maxavg_demand[p],
                 perturb_norm=env.demand_perturb_norm[p]) for p in range(P)]


def _capture_init(mod):
    """Wrap SupplyChainEnv.__init__ to record the nodes_info/kwargs the factories pass."""
    base = mod.SupplyChainEnv
    orig = base.__init__
    seen = {}

    def wrapped(self, nodes_info, **kw):
        seen["nodes_info"] = json.loads(json.dumps(nodes_info))
        seen["kwargs"] = dict(kw)
        orig(self, nodes_info, **kw)

    base.__init__ = wrapped
    return seen, lambda: setattr(base, "__init__", orig)


def _actions(kind, rng, T, n):
    if kind == "uniform":
        return rng.uniform(-1, 1, size=(T, n)).astype(np.float32)
    grid = np.array([-1.0, -0.5, 0.0, 0.25, 0.5, 1.0], dtype=np.float32)
    a = rng.uniform(-1.4, 1.4, size=(T, n)).astype(np.float32)
    mask = rng.uniform(size=(T, n)) < 0.5
    a[mask] = grid[rng.randint(0, len(grid), size=mask.sum())]
    return a


def _heap_arrays(env, H):
    nodes = env.nodes
    P = env.num_products
    t = np.full((len(nodes), P, H), -1, dtype=np.int32)
    v = np.zeros((len(nodes), P, H), dtype=np.float64)
    k = np.full((len(nodes), P, H), -1, dtype=np.int8)
    for i, nd in enumerate(nodes):
        for p, heap in enumerate(nd.shipments_by_prod):
            assert len(heap) <= H, "heap capacity"
            for j, (when, amount) in enumerate(heap):
                t[i, p, j] = int(when)
                v[i, p, j] = float(amount)
                k[i, p, j] = KIND[type(amount)]
    return t, v, k


def run_case(name, spec):
    import gym_supplychain.envs as envs
    from gym_supplychain.envs import supplychain_env as scmod
    seen, restore = _capture_init(scmod)
    try:
        env = getattr(envs, spec["factory"])(**spec["kwargs"])
    finally:
        restore()
    T = env.total_time_steps
    R = len(env.last_level_nodes)
    P = env.num_products
    n_act = env.action_space.shape[0]
    n_obs = env.observation_space.shape[0]
    n_lt = env.count_leadtimes_per_timestep if env.stochastic_leadtimes else 0
    N = spec["n_envs"]
    H = 64
    rng = np.random.RandomState(spec["seed"])
    seed = 1000 + spec["seed"]
    models = demand_models(env)
    rec = dict(obs=np.zeros((T + 1, N, n_obs)), reward=np.zeros((T, N)),
               stock=np.zeros((T + 1, N, len(env.nodes), P)),
               heap_t=np.zeros((T + 1, N, len(env.nodes), P, H), dtype=np.int32),
               heap_v=np.zeros((T + 1, N, len(env.nodes), P, H)),
               heap_k=np.zeros((T + 1, N, len(env.nodes), P, H), dtype=np.int8),
               actions=np.zeros((T, N, n_act), dtype=np.float32),
               demands=np.zeros((N, T + 1, R, P), dtype=np.int64),
               leadtimes=np.zeros((N, T, max(n_lt, 1)), dtype=np.int64))
    # build_info on (the factories do not forward it): env and nodes keep the per-episode
    # ledgers of info['sc_episode'] (:214-218, :684-695, :750-760); nothing else changes
    env.build_info = True
    for nd in env.nodes:
        nd.build_info = True
    nk = len(LEDGER_KEYS)
    for key, dt in (("led_cost", np.float64), ("led_units", np.float64)):
        rec[key] = np.zeros((T, N, nk, P), dtype=dt)
        rec[key + "_k"] = np.zeros((T, N, nk, P), dtype=np.int8)
    rec["led_rewards"] = np.zeros((T, N))
    for n in range(N):
        env.seed(n)
        env.reset()
        if all(m["std"] is None and m["sen_peaks"] is None for m in models) and not env.demand_config_by_product:
            dem = sc_demand_table(seed, n, 0, T, R, P, models[0]["lo"], models[0]["hi"])
        else:
            dem = sc_demand_table_models(seed, n, 0, T, R, P, models)
        # by product the reference keeps one (T+1, R) table per product (:655-661)
        env.customer_demands = [dem[:, :, p].copy() for p in range(P)] if env.demand_config_by_product else dem.copy()
        rec["demands"][n] = dem
        if n_lt:
            lts = sc_leadtime_table(seed, n, 0, T, n_lt, env.avg_leadtime, env.max_leadtime)
            env.leadtimes = lts.copy()
            rec["leadtimes"][n] = lts
        rec["obs"][0, n] = env._build_observation()
        rec["stock"][0, n] = [np.asarray(nd.stock, dtype=np.float64) for nd in env.nodes]
        rec["heap_t"][0, n], rec["heap_v"][0, n], rec["heap_k"][0, n] = _heap_arrays(env, H)
        acts = _actions(spec["act"], rng, T, n_act)
        rec["actions"][:, n] = acts
        for t in range(T):
            obs, r, done, info = env.step(acts[t].copy())
            assert done == (t == T - 1)
            rec["obs"][t + 1, n] = obs
            rec["reward"][t, n] = r
            rec["stock"][t + 1, n] = [np.asarray(nd.stock, dtype=np.float64) for nd in env.nodes]
            rec["heap_t"][t + 1, n], rec["heap_v"][t + 1, n], rec["heap_k"][t + 1, n] = _heap_arrays(env, H)
            led = info["sc_episode"]
            rec["led_rewards"][t, n] = float(led["rewards"])
            for j, key in enumerate(LEDGER_KEYS):
                for p in range(P):
                    for part, name in (("costs", "led_cost"), ("units", "led_units")):
                        x = led[part][key][p]
                        rec[name][t, n, j, p] = float(x)
                        rec[name + "_k"][t, n, j, p] = KIND[type(x)]
    used = int((rec["heap_t"] >= 0).sum(axis=-1).max())
    for k in ("heap_t", "heap_v", "heap_k"):
        rec[k] = rec[k][..., :max(used, 1)]
    meta = dict(factory=spec["factory"], factory_kwargs=spec["kwargs"], nodes_info=seen["nodes_info"],
                kwargs=seen["kwargs"], demand_models=models, T=T, R=R, P=P, n_act=n_act, n_obs=n_obs, n_lt=n_lt, seed=seed,
                node_names=[nd.label for nd in env.nodes])
    return rec, meta


def main():
    if not os.path.isdir(os.path.join(REFERENCE, "gym_supplychain")):
        print("gen_golden_sc: /root/reference absent; keeping committed fixtures")
        return 0
    sys.path.insert(0, REFERENCE)
    sys.path.insert(0, os.path.join(HERE, "refharness"))
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[1:]
    for name, spec in CASES.items():
        if only and name not in only:
            continue
        rec, meta = run_case(name, spec)
        path = os.path.join(OUT, f"sc_{name}.npz")
        np.savez_compressed(path, meta=np.array(json.dumps(meta)), **rec)
        print(f"wrote {path} ({os.path.getsize(path)} B) heap cap used {rec['heap_t'].shape[-1]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
