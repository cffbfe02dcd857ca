"""Helpers to read tests/golden/beergame_*.npz (written by oracle/gen_golden.py)."""
import glob
import os

import numpy as np

from conftest import GOLDEN


def beergame_cases():
    return sorted(os.path.basename(p)[len("beergame_"):-4] for p in glob.glob(os.path.join(GOLDEN, "beergame_*.npz")))


def load_beergame(name):
    g = dict(np.load(os.path.join(GOLDEN, f"beergame_{name}.npz")))
    L = int(g["levels"])
    info = dict(levels=L, inv_cost=int(g["inv_cost"]), backlog_cost=int(g["backlog_cost"]),
                initial_inventory=g["initial_inventory"].tolist(),
                initial_shipment_value=int(g["initial_shipment_value"]),
                initial_orders_value=int(g["initial_orders_value"]),
                shipment_delays=g["shipment_delays"].tolist())
    g["info"] = info
    g["is_poisson"] = float(g["lam"]) >= 0
    return g


# ---- SupplyChain (written by oracle/gen_golden_sc.py) ----------------------------------
SC_ORACLE_KW = ("num_products", "unmet_demand_cost", "exceeded_stock_capacity_cost", "exceeded_process_capacity_cost",
                "exceeded_ship_capacity_cost", "demand_range", "processing_ratio", "stochastic_leadtimes",
                "avg_leadtime", "max_leadtime", "total_time_steps", "demand_config_by_product")


def sc_cases():
    return sorted(os.path.basename(p)[len("sc_"):-4] for p in glob.glob(os.path.join(GOLDEN, "sc_*.npz")))


def load_sc(name):
    import json
    g = dict(np.load(os.path.join(GOLDEN, f"sc_{name}.npz")))
    g["meta"] = json.loads(str(g["meta"]))
    g["oracle_kwargs"] = {k: g["meta"]["kwargs"][k] for k in SC_ORACLE_KW if k in g["meta"]["kwargs"]}
    return g


# ---- BeerGameEnv2 (written by oracle/gen_golden_bg2.py) --------------------------------
def beergame2_cases():
    return sorted(os.path.basename(p)[len("beergame2_"):-4] for p in glob.glob(os.path.join(GOLDEN, "beergame2_*.npz")))


def load_beergame2(name):
    import ast
    g = dict(np.load(os.path.join(GOLDEN, f"beergame2_{name}.npz")))
    g["kwargs"] = ast.literal_eval(str(g["kwargs"]))
    return g


# ---- reference pins and RandomState fixtures (written by oracle/gen_golden_pins.py) ------
def load_ref_pins():
    """{case: dict(meta..., rewards=[T] float64, first_actions=[2, A] float32)}"""
    import json
    z = np.load(os.path.join(GOLDEN, "ref_pins.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    for name, m in meta.items():
        m["rewards"] = z[f"{name}/rewards"]
        m["first_actions"] = z[f"{name}/first_actions"]
    return meta


def load_ref_tables():
    """{fixture name: int64 array as stored in the reference's tests/data/<name>.npy}"""
    import json
    z = np.load(os.path.join(GOLDEN, "ref_tables.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    return {k: z[k].astype(np.int64) for k in meta}, meta
