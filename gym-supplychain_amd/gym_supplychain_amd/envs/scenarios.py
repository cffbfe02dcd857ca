"""The reference's scenario classes: nodes_info builders + SupplyChainEnv subclasses.

Config-only code in the reference: supplychain_2perstage_env.py,
supplychain_Nperstage_env.py, supplychain_multiproduct_env.py. Each builder returns the
nodes_info dict the reference's class hands to SupplyChainEnv.__init__ (checked equal
against the dicts captured from the reference in tests/golden/sc_*.npz), and each class
keeps the reference's keyword defaults. `*_nodes()` + `scenario_kwargs()` also feed
SupplyChainVecEnv (gym_supplychain_amd.make_vec).
"""
from .supplychain_env import SupplyChainEnv

_ENV_KEYS = ("num_products", "unmet_demand_cost", "exceeded_stock_capacity_cost", "exceeded_process_capacity_cost",
             "exceeded_ship_capacity_cost", "processing_ratio", "demand_range", "demand_std", "demand_sen_peaks",
             "avg_demand_range", "total_time_steps", "stochastic_leadtimes", "avg_leadtime", "max_leadtime", "seed",
             "build_info", "demand_perturb_norm", "demand_config_by_product")


def _env_kwargs(kw):
    return {k: kw[k] for k in _ENV_KEYS if k in kw}


# ---- sc-2perstage-v0 (supplychain_2perstage_env.py:3-64) --------------------------------
TWO_PER_STAGE_DEFAULTS = dict(
    num_products=1, initial_stocks=[0] * 8, initial_supply=[[[60, 60]]] * 2,
    initial_shipments=[[[60, 60]]] * 2 + [[[20, 20]]] * 4, supply_capacities=[120, 150],
    processing_capacities=[300, 300], stock_capacities=[200, 300] * 4, ship_capacity=300, processing_ratio=3,
    processing_costs=[12, 10], stock_costs=[1] * 8, supply_costs=[6, 4], dest_cost=2, unmet_demand_cost=216,
    exceeded_stock_capacity_cost=10, exceeded_process_capacity_cost=10, exceeded_ship_capacity_cost=10,
    demand_range=(10, 20), demand_std=None, demand_sen_peaks=None, avg_demand_range=None,
    stochastic_leadtimes=False, avg_leadtime=2, max_leadtime=2, total_time_steps=360, seed=None, build_info=False,
    demand_perturb_norm=False)


def two_per_stage_nodes(**kw):
    c = dict(TWO_PER_STAGE_DEFAULTS, **kw)
    P = c["num_products"]
    stocks = c["initial_stocks"] or [0] * 8
    costs = [[c["dest_cost"]] * 2] * P
    caps = [c["ship_capacity"]] * 2
    stage = {}
    for i in range(2):
        stage[f"Supplier{i + 1}"] = dict(initial_stock=stocks[i], initial_supply=c["initial_supply"][i],
                                        stock_capacity=c["stock_capacities"][i], stock_cost=c["stock_costs"][i],
                                        supply_capacity=c["supply_capacities"][i], supply_cost=c["supply_costs"][i],
                                        destinations=["Factory1", "Factory2"], dest_costs=costs, ship_capacity=caps)
    for i in range(2):
        stage[f"Factory{i + 1}"] = dict(initial_stock=stocks[2 + i], initial_shipments=c["initial_shipments"][i],
                                       stock_capacity=c["stock_capacities"][2 + i], stock_cost=c["stock_costs"][2 + i],
                                       processing_capacity=c["processing_capacities"][i],
                                       processing_cost=c["processing_costs"][i],
                                       destinations=["WholeSaler1", "WholeSaler2"], dest_costs=costs, ship_capacity=caps)
    for i in range(2):
        stage[f"WholeSaler{i + 1}"] = dict(initial_stock=stocks[4 + i], initial_shipments=c["initial_shipments"][2 + i],
                                          stock_capacity=c["stock_capacities"][4 + i],
                                          stock_cost=c["stock_costs"][4 + i],
                                          destinations=["Retailer1", "Retailer2"], dest_costs=costs, ship_capacity=caps)
    for i in range(2):
        stage[f"Retailer{i + 1}"] = dict(initial_stock=stocks[6 + i], initial_shipments=c["initial_shipments"][4 + i],
                                        stock_capacity=c["stock_capacities"][6 + i], stock_cost=c["stock_costs"][6 + i],
                                        last_level=True)
    return stage, _env_kwargs(c)


# ---- sc-2perstage-seasonal-v0 (supplychain_2perstage_env.py:67-97) ------------------------
SEASONAL_DEFAULTS = dict(
    TWO_PER_STAGE_DEFAULTS, initial_stocks=[800] * 8, initial_supply=[[[600, 600]], [[840, 840]]],
    initial_shipments=[[[600, 600]], [[840, 840]]] + [[[240, 240]]] * 4, supply_capacities=[600, 840],
    processing_capacities=[840, 960], stock_capacities=[1600, 1800] * 4, ship_capacity=1800,
    demand_range=(0, 400), demand_std=10, demand_sen_peaks=4, avg_demand_range=(150, 250), demand_perturb_norm=True)


def two_per_stage_seasonal_nodes(check_actions=False, **kw):
    return two_per_stage_nodes(**dict(SEASONAL_DEFAULTS, **kw))


# ---- sc-Nperstage-multiproduct-v0 / ntom (supplychain_Nperstage_env.py:3-131) -------------
N_PER_STAGE_DEFAULTS = dict(
    nodes_per_echelon=3, num_products=2, initial_stocks=None, stock_capacities=None, stock_costs=1,
    initial_supply=None, supply_capacities=None, supply_costs=None, dest_cost=None, ship_capacity=None,
    initial_shipments=None, processing_capacities=None, processing_costs=None, processing_ratio=3,
    unmet_demand_cost=216, exceeded_stock_capacity_cost=10, exceeded_process_capacity_cost=10,
    exceeded_ship_capacity_cost=10, demand_range=(0, 400), demand_std=None, demand_sen_peaks=None,
    avg_demand_range=None, demand_perturb_norm=False, stochastic_leadtimes=False, avg_leadtime=2, max_leadtime=2,
    total_time_steps=360, seed=None, build_info=False)

ECHELONS = ("suppliers", "factories", "wholesalers", "retailers")


def n_per_stage_nodes(**kw):
    c = dict(N_PER_STAGE_DEFAULTS, **kw)
    P, lt = c["num_products"], c["avg_leadtime"]
    npe = c["nodes_per_echelon"]
    if isinstance(npe, int):
        npe = [npe] * 4
    n = dict(zip(ECHELONS, npe))
    stock_caps = c["stock_capacities"] or {
        "suppliers": [[1600] * P] * n["suppliers"], "factories": [[6400] * P] * n["factories"],
        "wholesalers": [[1600] * P] * n["wholesalers"], "retailers": [[1600] * P] * n["retailers"]}
    init_stocks = c["initial_stocks"] or {e: [[800] * P] * n[e] for e in ECHELONS}
    init_supply = c["initial_supply"] or [[[600] * lt] * P] * n["suppliers"]
    supply_caps = c["supply_capacities"] or [[600] * P] * n["suppliers"]
    supply_costs = c["supply_costs"] or [[6] * P] * n["suppliers"]
    dest_cost = c["dest_cost"] or {"suppliers": [[2] * n["factories"]] * P,
                                   "factories": [[2] * n["wholesalers"]] * P,
                                   "wholesalers": [[2] * n["retailers"]] * P}
    ship_cap = c["ship_capacity"] or {"suppliers": [500 * P] * n["factories"],
                                      "factories": [500 * P] * n["wholesalers"],
                                      "wholesalers": [500 * P] * n["retailers"]}
    init_ship = c["initial_shipments"] or {"factories": [[[600] * lt] * P] * n["factories"],
                                           "wholesalers": [[[240] * lt] * P] * n["wholesalers"],
                                           "retailers": [[[240] * lt] * P] * n["retailers"]}
    proc_caps = c["processing_capacities"] or [840 * P] * n["factories"]
    proc_costs = c["processing_costs"] or [[12] * P] * n["factories"]
    stock_cost = c["stock_costs"]
    nodes = {}
    for i in range(n["suppliers"]):
        nodes[f"Supplier{i}"] = dict(initial_stock=init_stocks["suppliers"][i],
                                     stock_capacity=stock_caps["suppliers"][i], stock_cost=stock_cost,
                                     initial_supply=init_supply[i], supply_capacity=supply_caps[i],
                                     supply_cost=supply_costs[i],
                                     destinations=[f"Factory{j}" for j in range(n["factories"])],
                                     dest_costs=dest_cost["suppliers"], ship_capacity=ship_cap["suppliers"])
    for i in range(n["factories"]):
        nodes[f"Factory{i}"] = dict(initial_stock=init_stocks["factories"][i],
                                    stock_capacity=stock_caps["factories"][i], stock_cost=stock_cost,
                                    initial_shipments=init_ship["factories"][i],
                                    processing_capacity=proc_caps[i], processing_cost=proc_costs[i],
                                    destinations=[f"Wholesal{j}" for j in range(n["wholesalers"])],
                                    dest_costs=dest_cost["factories"], ship_capacity=ship_cap["factories"])
    for i in range(n["wholesalers"]):
        nodes[f"Wholesal{i}"] = dict(initial_stock=init_stocks["wholesalers"][i],
                                     stock_capacity=stock_caps["wholesalers"][i], stock_cost=stock_cost,
                                     initial_shipments=init_ship["wholesalers"][i],
                                     destinations=[f"Retailer{j}" for j in range(n["retailers"])],
                                     dest_costs=dest_cost["wholesalers"], ship_capacity=ship_cap["wholesalers"])
    for i in range(n["retailers"]):
        nodes[f"Retailer{i}"] = dict(initial_stock=init_stocks["retailers"][i],
                                     stock_capacity=stock_caps["retailers"][i], stock_cost=stock_cost,
                                     initial_shipments=init_ship["retailers"][i], last_level=True)
    return nodes, _env_kwargs(c)


# ---- sc-2perstage-multiproduct-v0 (supplychain_multiproduct_env.py:3-114) ---------------
MULTI_PRODUCT_DEFAULTS = dict(
    demand_config_by_product=False, num_products=2, initial_stocks=None, stock_capacities=None, stock_costs=1,
    initial_supply=None, supply_capacities=None, supply_costs=None, dest_cost=None, ship_capacity=None,
    initial_shipments=None, processing_capacities=None, processing_costs=None, processing_ratio=3,
    unmet_demand_cost=216, exceeded_stock_capacity_cost=10, exceeded_process_capacity_cost=10,
    exceeded_ship_capacity_cost=10, demand_range=(0, 400), demand_std=None, demand_sen_peaks=None,
    avg_demand_range=None, demand_perturb_norm=False, stochastic_leadtimes=False, avg_leadtime=2, max_leadtime=2,
    total_time_steps=360, seed=None, build_info=False)


def multi_product_nodes(**kw):
    c = dict(MULTI_PRODUCT_DEFAULTS, **kw)
    P, lt = c["num_products"], c["avg_leadtime"]
    stock_caps = c["stock_capacities"] or [[1600] * P, [1800] * P, [6400] * P, [7200] * P,
                                           [1600] * P, [1800] * P, [1600] * P, [1800] * P]
    init_stocks = c["initial_stocks"] or [[800] * P] * 8
    init_supply = c["initial_supply"] or [[[600] * lt] * P, [[840] * lt] * P]
    supply_caps = c["supply_capacities"] or [[600] * P, [840] * P]
    supply_costs = c["supply_costs"] or [[6] * P, [4] * P]
    dest_cost = c["dest_cost"] or [[2] * 2] * P
    ship_cap = c["ship_capacity"] or [500 * P, 500 * P]
    init_ship = c["initial_shipments"] or ([[[600] * lt] * P, [[840] * lt] * P] + [[[240] * lt] * P] * 4)
    proc_caps = c["processing_capacities"] or [840 * P, 960 * P]
    proc_costs = c["processing_costs"] or [[12] * P, [10] * P]
    sc = c["stock_costs"]
    nodes = {}
    for i in range(2):
        nodes[f"Supplier{i + 1}"] = dict(initial_stock=init_stocks[i], stock_capacity=stock_caps[i], stock_cost=sc,
                                        initial_supply=init_supply[i], supply_capacity=supply_caps[i],
                                        supply_cost=supply_costs[i], destinations=["Factory1", "Factory2"],
                                        dest_costs=dest_cost, ship_capacity=ship_cap)
    for i in range(2):
        nodes[f"Factory{i + 1}"] = dict(initial_stock=init_stocks[2 + i], stock_capacity=stock_caps[2 + i],
                                       stock_cost=sc, initial_shipments=init_ship[i],
                                       processing_capacity=proc_caps[i], processing_cost=proc_costs[i],
                                       destinations=["Wholesal1", "Wholesal2"], dest_costs=dest_cost,
                                       ship_capacity=ship_cap)
    for i in range(2):
        nodes[f"Wholesal{i + 1}"] = dict(initial_stock=init_stocks[4 + i], stock_capacity=stock_caps[4 + i],
                                        stock_cost=sc, initial_shipments=init_ship[2 + i],
                                        destinations=["Retailer1", "Retailer2"], dest_costs=dest_cost,
                                        ship_capacity=ship_cap)
    for i in range(2):
        nodes[f"Retailer{i + 1}"] = dict(initial_stock=init_stocks[6 + i], stock_capacity=stock_caps[6 + i],
                                        stock_cost=sc, initial_shipments=init_ship[4 + i], last_level=True)
    return nodes, _env_kwargs(c)


def increasing_costs_kwargs(num_products=2, **kw):
    """SupplyChainMultiProduct_IncreasingCosts (supplychain_multiproduct_env.py:117-155)."""
    P = num_products
    return dict(kw, num_products=P,
                supply_costs=[[6 * (i + 1) for i in range(P)], [4 * (i + 1) for i in range(P)]],
                dest_cost=[[2 * (i + 1)] * 2 for i in range(P)],
                processing_costs=[[12 * (i + 1) for i in range(P)], [10 * (i + 1) for i in range(P)]],
                stock_costs=[1 * (i + 1) for i in range(P)])


def by_product_demand_kwargs(num_products=2, demand_std=None, demand_perturb_norm=False, inc_costs=False, **kw):
    """SupplyChainMultiProduct_DemConfigByProd(_IncCosts) (supplychain_multiproduct_env.py:157-274):
    product 1 seasonal (0..400, 4 peaks, mean 100..300), product 2 regular (0..300),
    product 3 seasonal (0..400, 2 peaks); at most 3 products."""
    P = num_products
    if not 1 <= P <= 3:
        raise AssertionError("at most 3 products (supplychain_multiproduct_env.py:174)")
    # the _IncCosts variant appends [demand_std] (a list) for products 2 and 3 (:243, :250)
    later_std = [demand_std] if inc_costs else demand_std
    ranges, stds, peaks, avg = [(0, 400)], [demand_std], [4], [(100, 300)]
    if P > 1:
        ranges.append((0, 300)), stds.append(later_std), peaks.append(None), avg.append(None)
    if P > 2:
        ranges.append((0, 400)), stds.append(later_std), peaks.append(2), avg.append((100, 300))
    out = dict(kw, num_products=P, demand_config_by_product=True, demand_range=ranges, demand_std=stds,
               demand_sen_peaks=peaks, avg_demand_range=avg, demand_perturb_norm=[demand_perturb_norm] * P)
    return increasing_costs_kwargs(**out) if inc_costs else out


SCENARIOS = {
    "sc-2perstage-v0": two_per_stage_nodes,
    "sc-Nperstage-multiproduct-v0": n_per_stage_nodes,
    "sc-2perstage-multiproduct-v0": multi_product_nodes,
    "sc-2perstage-multiproduct-inccosts-v0": lambda **kw: multi_product_nodes(**increasing_costs_kwargs(**kw)),
    "sc-2perstage-seasonal-v0": two_per_stage_seasonal_nodes,
    "sc-2perstage-multiproduct-v1": lambda **kw: multi_product_nodes(**by_product_demand_kwargs(**kw)),
    "sc-2perstage-multiproduct-inccosts-v1":
        lambda **kw: multi_product_nodes(**by_product_demand_kwargs(inc_costs=True, **kw)),
}


class _Scenario(SupplyChainEnv):
    _builder = None

    def __init__(self, device=None, **kw):
        nodes, env_kw = type(self)._builder(**kw)
        super().__init__(nodes, device=device, **env_kw)


class SupplyChain2perStageEnv(_Scenario):
    """sc-2perstage-v0: 2 suppliers, 2 factories, 2 wholesalers, 2 retailers."""
    _builder = staticmethod(two_per_stage_nodes)


class SupplyChainNPerStage(_Scenario):
    """N per echelon, fully connected; ntom = SupplyChainNPerStage(nodes_per_echelon=[8, 8, 8, 16])."""
    _builder = staticmethod(n_per_stage_nodes)


class SupplyChainMultiProduct(_Scenario):
    _builder = staticmethod(multi_product_nodes)


class SupplyChainMultiProduct_IncreasingCosts(_Scenario):
    _builder = staticmethod(lambda **kw: multi_product_nodes(**increasing_costs_kwargs(**kw)))


class SupplyChain2perStageSeasonalEnv(_Scenario):
    """sc-2perstage-seasonal-v0: 2-per-stage chain, sinusoidal demand with normal perturbation."""
    _builder = staticmethod(two_per_stage_seasonal_nodes)


class SupplyChainMultiProduct_DemConfigByProd(_Scenario):
    """sc-2perstage-multiproduct-v1: demand configured per product."""
    _builder = staticmethod(lambda **kw: multi_product_nodes(**by_product_demand_kwargs(**kw)))


class SupplyChainMultiProduct_DemConfigByProd_IncCosts(_Scenario):
    """sc-2perstage-multiproduct-inccosts-v1: per-product demand and increasing costs."""
    _builder = staticmethod(lambda **kw: multi_product_nodes(**by_product_demand_kwargs(inc_costs=True, **kw)))
