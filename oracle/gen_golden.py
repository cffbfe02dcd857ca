"""Generate tests/golden/beergame_*.npz from the REFERENCE itself — build container only.

Runs the real gym_supplychain BeerGameEnv (imported read-only from /root/reference with
the inert gym stand-in under oracle/refharness/, see its docstring) one env at a time,
driven by explicit integer actions and by per-env customer_demand lists drawn with the
oracle's Philox4x32-10 + Poisson inversion (oracle/philox.py, oracle/poisson.py) — the
same draws the HIP kernel makes on device. Nothing is written under /root/reference
(bytecode writing is disabled). On a machine without /root/reference this script exits
cleanly without touching tests/golden/.

    python oracle/gen_golden.py [case ...] # rewrites tests/golden/beergame_*.npz (or those cases)
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
from oracle.philox import STREAM_DEMAND, draw_words  # noqa: E402
from oracle.poisson import poisson_invert, poisson_thresholds  # noqa: E402

# Each case: env_init_info shared by all envs (delays/costs/levels are env config),
# per-env Poisson demand (or the fixed list), and an action generator.
CASES = {
    # BASELINE config 2 semantics at golden size: defaults + Poisson(8) demand
    "default_poisson": dict(info={}, n_envs=64, weeks=35, lam=8.0, seed=0x5EED0000, episode=0,
                            act_range=(0, 8), act_seed=0),
    # delay-0 weeks (direct delivery, :93-94/:111-112), negative actions (F4), costs, init values
    "vardelay_negact": dict(info=dict(inv_cost=3, backlog_cost=5, initial_inventory=[10, 12, 14, 16],
                                      initial_shipment_value=5, initial_orders_value=6),
                            delays=("randint", 1, 0, 4), n_envs=64, weeks=35, lam=8.0, seed=1, episode=0,
                            act_range=(-4, 4), act_seed=1),
    # colliding targets (several weeks shipping into one arrival week) and a deep pipeline
    "delay_collide": dict(info=dict(), delays=("pattern", [6, 5, 4, 3, 2, 1, 0, 3, 1, 6, 2, 2, 5, 0, 1]),
                          n_envs=32, weeks=30, lam=12.0, seed=7, episode=3, act_range=(-2, 10), act_seed=2),
    # 3-level chain, the reference's fixed default demand list
    "levels3_fixed": dict(info=dict(levels=3, initial_inventory=[12, 12, 12]), n_envs=16, weeks=35,
                          lam=None, seed=0, episode=0, act_range=(0, 8), act_seed=3),
    # 6-level chain, short horizon, second episode counter
    "levels6_short": dict(info=dict(levels=6, initial_inventory=[12, 9, 15, 12, 20, 3], inv_cost=2,
                                    backlog_cost=7),
                          n_envs=32, weeks=20, lam=4.5, seed=123456789012, episode=1,
                          act_range=(-3, 6), act_seed=4),
    # 1-level chain edge case (incoming[1:] / [:-1] slices are empty)
    "levels1": dict(info=dict(levels=1, initial_inventory=[5]), n_envs=8, weeks=12, lam=3.0, seed=9,
                    episode=0, act_range=(0, 5), act_seed=5),
    # a 150-week horizon with delays up to 70: the reference's table has 222
    # rows (:46-50), past the state slab's 127, and rows past the horizon are written
    "long_delay70": dict(info=dict(), delays=("pattern", [70, 3, 0, 12, 70, 1, 45, 2, 0, 70, 6, 33]),
                         n_envs=4, weeks=150, lam=8.0, seed=31, episode=0, act_range=(-3, 12), act_seed=6),
}


def case_inputs(name, spec):
    info = dict(spec["info"])
    T = spec["weeks"]
    L = info.get("levels", 4)
    N = spec["n_envs"]
    env_ids = np.arange(N, dtype=np.uint64)
    if spec["lam"] is None:
        base = [4] * 4 + [8] * 31
        demand = np.tile(np.asarray(base[:T], dtype=np.int64), (N, 1))
        thr = np.zeros(0, dtype=np.uint32)
    else:
        thr = poisson_thresholds(spec["lam"])
        words = draw_words(spec["seed"], env_ids, spec["episode"], T, STREAM_DEMAND)
        demand = poisson_invert(words, thr).astype(np.int64)
    if "delays" in spec:
        kind = spec["delays"][0]
        if kind == "randint":
            _, s, lo, hi = spec["delays"]
            delays = np.random.RandomState(s).randint(lo, hi, size=T).tolist()
        else:
            pat = spec["delays"][1]
            delays = [pat[i % len(pat)] for i in range(T)]
        info["shipment_delays"] = [int(d) for d in delays]
    lo, hi = spec["act_range"]
    actions = np.random.RandomState(spec["act_seed"]).randint(lo, hi + 1, size=(T, N, L)).astype(np.int64)
    return info, demand, actions, thr


SHIP_ENVS = 8


def run_reference(info, demand, actions):
    from gym_supplychain.envs import BeerGameEnv
    T, N, L = actions.shape
    rec = {k: np.zeros((T, N, L), dtype=np.int64) for k in ("obs", "inventory", "backlog", "orders_placed")}
    rec["reward"] = np.zeros((T, N), dtype=np.int64)
    rec["done"] = np.zeros((T, N), dtype=bool)
    rec["reset_obs"] = np.zeros((N, L), dtype=np.int64)
    rec["inventory_costs"] = np.zeros((N, L), dtype=np.int64)
    rec["backlog_costs"] = np.zeros((N, L), dtype=np.int64)
    rec["all_orders_placed"] = np.zeros((N, L, T + 1), dtype=np.int64)
    rec["past_horizon_raises"] = np.zeros(N, dtype=bool)
    # the order slips of every week, and the whole absolute-week shipment table of the
    # first SHIP_ENVS envs every week (beergame_env.py:46-52, :79-81)
    rec["incoming_orders"] = np.zeros((T, N, L), dtype=np.int64)
    ns = min(N, SHIP_ENVS)
    rec["shipments"] = None
    for n in range(N):
        env_info = dict(info)
        env_info["customer_demand"] = [int(x) for x in demand[n]]
        env = BeerGameEnv(env_info)
        rec["reset_obs"][n] = env.reset()
        for w in range(T):
            obs, r, done, extra = env.step(actions[w, n])
            assert extra == {} and isinstance(r, np.integer)
            rec["obs"][w, n] = obs
            rec["reward"][w, n] = r
            rec["done"][w, n] = done
            rec["inventory"][w, n] = env.inventory
            rec["backlog"][w, n] = env.backlog
            rec["orders_placed"][w, n] = env.orders_placed
            rec["incoming_orders"][w, n] = env.incoming_orders
            if n < ns:
                if rec["shipments"] is None:
                    rec["shipments"] = np.zeros((T, ns) + env.shipments.shape, dtype=np.int64)
                rec["shipments"][w, n] = env.shipments
        rec["inventory_costs"][n] = env.inventory_costs
        rec["backlog_costs"][n] = env.backlog_costs
        rec["all_orders_placed"][n] = env.all_orders_placed
        try:
            env.step(actions[0, n])
        except IndexError:
            rec["past_horizon_raises"][n] = True
    return rec


def main():
    if not os.path.isdir(os.path.join(REFERENCE, "gym_supplychain")):
        print("gen_golden: /root/reference absent; keeping committed fixtures")
        return 0
    sys.path.insert(0, REFERENCE)
    sys.path.insert(0, os.path.join(HERE, "refharness"))
    os.makedirs(OUT, exist_ok=True)
    only = set(sys.argv[1:])  # case names to (re)write; all by default
    for name, spec in CASES.items():
        if only and name not in only:
            continue
        info, demand, actions, thr = case_inputs(name, spec)
        rec = run_reference(info, demand, actions)
        T, N, L = actions.shape
        delays = info.get("shipment_delays", [2] * T)
        payload = dict(
            levels=np.int32(L), weeks=np.int32(T), n_envs=np.int32(N),
            inv_cost=np.int32(info.get("inv_cost", 1)), backlog_cost=np.int32(info.get("backlog_cost", 2)),
            initial_inventory=np.asarray(info.get("initial_inventory", [12] * 4), dtype=np.int32),
            initial_shipment_value=np.int32(info.get("initial_shipment_value", 4)),
            initial_orders_value=np.int32(info.get("initial_orders_value", 4)),
            shipment_delays=np.asarray(delays, dtype=np.int32),
            lam=np.float64(-1.0 if spec["lam"] is None else spec["lam"]),
            seed=np.uint64(spec["seed"]), episode=np.uint32(spec["episode"]),
            poisson_thresholds=thr,
            demand=demand.astype(np.int32), actions=actions.astype(np.int32),
        )
        for k, v in rec.items():
            payload["ref_" + k] = v.astype(np.int32) if v.dtype == np.int64 else v
        path = os.path.join(OUT, f"beergame_{name}.npz")
        np.savez_compressed(path, **payload)
        print(f"wrote {path}: N={N} T={T} L={L} ({os.path.getsize(path)} B)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
