"""Generic multi-echelon supply chain on MI355X: ``SupplyChainVecEnv`` and the drop-in
``SupplyChainEnv`` plus the reference's scenario classes.

Mirrors gym_supplychain.envs.SupplyChainEnv (gym_supplychain/envs/supplychain_env.py,
snapshot 2024-08-07): same nodes_info schema and constructor keywords (:482-628), same
reset()/step() results (:630-748). The dynamics — SC_Node.act with SC_Action.apply, the
heapq in-transit pipeline, the observation walk over heap storage order — run in
gym-supplychain_amd/csrc/scg_supplychain.hip through include/scgpu.h; this module
resolves the configuration into the flat node table the kernels read and owns the
device buffers.

Differences from the reference:
  * per-episode demand and stochastic lead times are drawn on device with Philox (same
    distributions: uniform / normal / sinusoidal demand per product (envs/demand.py),
    clip(1 + Poisson(avg-1), 1, max) lead times) instead of MT19937 RandomState, keyed by
    `seed` and the global env id; caller tables replay any host draw exactly;
  * actions are float32 (the declared Box dtype); the vec env's observations are float32
    by default (float64, the reference's dtype, on request and in the single-env class);
  * build_info=True keeps info['sc_episode'] on the device (lane and staged kernels); the
    drop-in env returns it with the reference's per-entry NumPy types.
"""
import atexit
import ctypes
import hashlib
import os
import weakref

import numpy as np
import torch

from .. import _native as nat
from .. import checkpoint as ckpt
from .. import spaces
from . import demand
from . import resident
from ..distributed import entropy_seed

_MAXP = nat.SC_MAX_PRODUCTS
_MAXD = nat.SC_MAX_DESTS
_MAXI = nat.SC_MAX_INIT


def _per_product(value, P, what):
    """SC_Node._treat_int_or_list_param (:178-191)."""
    if type(value) is list:
        if len(value) == 0:
            return [0] * P
        if len(value) != P:
            raise AssertionError(f"{what}: expected one value per product ({P}), got {len(value)}")
        return list(value)
    if type(value) is int:
        return [value] * P
    raise ValueError(f"Invalid param: '{value}' should be an int or a list with one value per product")


def _int(name, v):
    if isinstance(v, (bool, np.bool_)) or not isinstance(v, (int, np.integer)):
        raise TypeError(f"{name} must be an integer (got {v!r}); the GPU path keeps the reference's int costs")
    v = int(v)
    if abs(v) >= 2 ** 31:
        raise ValueError(f"{name}={v} does not fit int32")
    return v


# NumPy type codes of ledger entries (scg_npscalar.h NpKind) -> the reference's scalar types
_SC_TYPES = {0: lambda x: int(x), 1: float, 2: np.float32, 3: np.float64, 4: np.int64}


class SupplyChainSpec:
    """SupplyChainEnv.__init__ (:482-628) resolved into scg_sc_node records."""

    def __init__(self, nodes_info, num_products=1, unmet_demand_cost=1000, exceeded_stock_capacity_cost=1000,
                 exceeded_process_capacity_cost=1000, exceeded_ship_capacity_cost=1000,
                 demand_config_by_product=False, demand_range=(10, 20), demand_std=None, demand_sen_peaks=None,
                 avg_demand_range=None, processing_ratio=3, stochastic_leadtimes=False, avg_leadtime=2,
                 max_leadtime=2, total_time_steps=360, seed=None, build_info=False, demand_perturb_norm=False):
        self.build_info = bool(build_info)
        P = _int("num_products", num_products)
        if not 1 <= P <= _MAXP:
            raise ValueError(f"num_products={P} outside 1..{_MAXP}")
        self.P = P
        self.demand_config_by_product = bool(demand_config_by_product)
        ranges = list(demand_range) if demand_config_by_product else [demand_range] * P
        if len(ranges) != P:
            raise AssertionError("demand_range needs one (low, high) per product")
        for lo, hi in ranges:
            if lo == hi:
                raise AssertionError("demand_range must not be empty")  # :592-595
            if _int("demand_range[1]", hi) < _int("demand_range[0]", lo):
                raise ValueError("demand_range must be (low, high) with low < high")
        self.demand_range = tuple(ranges[0]) if not demand_config_by_product else [tuple(r) for r in ranges]
        # per-product generators (demands_generator.py:3-89; envs/demand.py)
        self.demand_models = demand.models_for(dict(
            demand_config_by_product=demand_config_by_product, demand_range=demand_range, demand_std=demand_std,
            demand_sen_peaks=demand_sen_peaks, avg_demand_range=avg_demand_range,
            demand_perturb_norm=demand_perturb_norm), P)
        self.penalties = dict(unmet_demand_cost=_int("unmet_demand_cost", unmet_demand_cost),
                              exceeded_stock_capacity_cost=_int("exceeded_stock_capacity_cost",
                                                                exceeded_stock_capacity_cost),
                              exceeded_process_capacity_cost=_int("exceeded_process_capacity_cost",
                                                                  exceeded_process_capacity_cost),
                              exceeded_ship_capacity_cost=_int("exceeded_ship_capacity_cost",
                                                               exceeded_ship_capacity_cost))
        self.stochastic_leadtimes = bool(stochastic_leadtimes)
        self.avg_leadtime = _int("avg_leadtime", avg_leadtime)
        self.max_leadtime = _int("max_leadtime", max_leadtime)
        self.total_time_steps = _int("total_time_steps", total_time_steps)
        self.seed = seed
        self.processing_ratio = processing_ratio
        names = list(nodes_info)
        if not 1 <= len(names) <= nat.SC_MAX_NODES:
            raise ValueError(f"{len(names)} nodes (1..{nat.SC_MAX_NODES} supported)")
        index = {n: i for i, n in enumerate(names)}
        self.node_names = names
        nodes = []
        for name in names:
            info = nodes_info[name]
            proc_cost = info.get("processing_cost", 0)
            no_proc = ((type(proc_cost) is int and proc_cost == 0) or
                       (type(proc_cost) is list and sum(proc_cost) == 0))           # :518-522
            supply_cap = _per_product(info.get("supply_capacity", 0), P, "supply_capacity")
            nd = dict(
                name=name,
                last_level=bool(info.get("last_level", False)),
                ratio=_per_product(0 if no_proc else processing_ratio, P, "processing_ratio"),
                processing_cost=_per_product(proc_cost, P, "processing_cost"),
                processing_capacity=info.get("processing_capacity", 0),
                supply_capacity=supply_cap if max(supply_cap) > 0 else [0] * P,
                supply_cost=_per_product(info.get("supply_cost", 0), P, "supply_cost"),
                max_ship=list(supply_cap) if max(supply_cap) > 0 else [0] * P,
                initial_stock=_per_product(info.get("initial_stock", 0), P, "initial_stock"),
                stock_capacity=_per_product(info.get("stock_capacity", float("inf")), P, "stock_capacity"),
                stock_cost=_per_product(info.get("stock_cost", 0), P, "stock_cost"),
                initial_supply=info.get("initial_supply", None),
                initial_shipments=info.get("initial_shipments", None),
                dests=[], ship_capacity=[], dest_costs=[[] for _ in range(P)],
            )
            nd["n_supply"] = sum(1 for c in nd["supply_capacity"] if c > 0)
            nodes.append(nd)
        for name in names:                                                            # define_destinations
            info = nodes_info[name]
            if "destinations" not in info:
                continue
            nd = nodes[index[name]]
            nd["dests"] = [index[d] for d in info["destinations"]]
            nd["ship_capacity"] = list(info["ship_capacity"])
            nd["dest_costs"] = [list(info["dest_costs"][p]) for p in range(P)]
            for i, d in enumerate(nd["dests"]):
                for p in range(P):
                    nodes[d]["max_ship"][p] += nd["ship_capacity"][i]
        a_off = lt_off = r_idx = 0
        for nd in nodes:
            nd["n_ship"] = sum(len(nd["dests"]) for p in range(P) if nd["stock_capacity"][p] > 0)
            nd["action_offset"], nd["leadtime_offset"] = a_off, lt_off
            a_off += nd["n_supply"] + nd["n_ship"]
            lt_off += (P if nd["n_supply"] > 0 else 0) + len(nd["dests"])
            nd["retailer_index"] = -1
            if nd["last_level"]:
                nd["retailer_index"] = r_idx
                r_idx += 1
        self.nodes = nodes
        self.n_retailers = r_idx
        self.n_actions = a_off
        self.n_leadtimes = lt_off
        self.n_obs = r_idx * P + len(nodes) * P + len(nodes) * P * self.avg_leadtime + 1      # :617-621

    def node_table(self):
        """The scg_sc_node array (host) for scg_sc_prepare and the device copy."""
        P = self.P
        table = (nat.ScNode * len(self.nodes))()
        for i, nd in enumerate(self.nodes):
            r = table[i]
            r.last_level = int(nd["last_level"])
            r.n_supply, r.n_ship, r.n_dests = nd["n_supply"], nd["n_ship"], len(nd["dests"])
            if r.n_dests > _MAXD:
                raise ValueError(f"node {nd['name']}: {r.n_dests} destinations (max {_MAXD})")
            r.processing_capacity = _int("processing_capacity", nd["processing_capacity"])
            r.retailer_index = nd["retailer_index"]
            r.action_offset, r.leadtime_offset = nd["action_offset"], nd["leadtime_offset"]
            for p in range(P):
                r.supply_capacity[p] = _int("supply_capacity", nd["supply_capacity"][p])
                r.supply_cost[p] = _int("supply_cost", nd["supply_cost"][p])
                r.stock_capacity[p] = _int("stock_capacity", nd["stock_capacity"][p])
                r.stock_cost[p] = _int("stock_cost", nd["stock_cost"][p])
                r.processing_ratio[p] = _int("processing_ratio", nd["ratio"][p])
                r.processing_cost[p] = _int("processing_cost", nd["processing_cost"][p])
                r.max_ship[p] = _int("max_ship", nd["max_ship"][p])
                r.initial_stock[p] = _int("initial_stock", nd["initial_stock"][p])
                k = 0
                for tbl in (nd["initial_supply"], nd["initial_shipments"]):                 # :405-412
                    if tbl:
                        for j, amount in enumerate(tbl[p]):
                            if k >= _MAXI:
                                raise ValueError(f"node {nd['name']}: more than {_MAXI} initial pipeline entries")
                            r.init_time[p][k] = j + 1
                            r.init_amount[p][k] = _int("initial pipeline amount", amount)
                            k += 1
                r.n_init[p] = k
                for i_d in range(len(nd["dests"])):
                    r.dest_costs[p][i_d] = _int("dest_costs", nd["dest_costs"][p][i_d])
            for i_d, d in enumerate(nd["dests"]):
                r.dests[i_d] = d
                r.ship_capacity[i_d] = _int("ship_capacity", nd["ship_capacity"][i_d])
        return table


def _default_seed(seed, seed_group=None):
    # RandomState(None) draws fresh entropy (:564); so do we (distributed.entropy_seed)
    return entropy_seed(seed, seed_group)


class SupplyChainVecEnv:
    """N lock-step SupplyChainEnv instances on one GPU.

    reset() -> obs [N, n_obs]
    step(actions float32 [N, n_actions] in [-1, 1]) -> (obs, reward float64 [N], done bool [N], info)

    Returned tensors are this env's output buffers (clone() to keep them). With
    auto_reset the terminal step resets every env in the same kernel; info then holds
    'terminal_observation' and 'episode_return'.

    demand_table / leadtime_table: optional device int32 tensors [N, T+1, R, P] /
    [N, T, n_lt] used for every episode instead of the Philox draws (e.g. to replay the
    reference's RandomState episodes exactly).
    kernel: "auto" / "lane" (one lane walks one env's whole chain), "level" (a lane group
    per env, one lane per node of a level), "staged" (one lane per env, the current
    node's heaps in LDS, shipments through an HBM inbox) or "nodes" (a wave per node of 64
    envs, every node acting at once, heaps and shipments in LDS; with build_info the lane
    kernel runs instead); DESIGN.md §6. All give the same results; the state layout follows
    the kernel.
    spec.build_info: every step's info holds 'sc_episode' = {'rewards': [N], 'costs':
    {key: [N, P]}, 'units': {key: [N, P]}} (device views, float64; the NumPy type of every
    entry in ledger_kinds()), the reference's episode ledgers (:684-695, :750-760); with
    auto-reset the terminal step adds 'terminal_sc_episode' for the finished episode.
    Every kernel but the level kernel (the node-parallel one keeps each node's entries of a
    step apart and adds them in node order, :750-760).
    """

    _KERNELS = {"auto": nat.SC_KERNEL_AUTO, "lane": nat.SC_KERNEL_LANE, "level": nat.SC_KERNEL_LEVEL,
                "staged": nat.SC_KERNEL_STAGED, "nodes": nat.SC_KERNEL_NODES}

    def __init__(self, n_envs, nodes_info=None, spec=None, seed=0, device=None, env_offset=0, auto_reset=True,
                 obs_dtype=torch.float32, track_returns=True, demand_table=None, leadtime_table=None, kernel="auto",
                 seed_group=None, **kwargs):
        if spec is None:
            if nodes_info is None:
                raise ValueError("pass nodes_info (+ SupplyChainEnv keywords) or a SupplyChainSpec")
            spec = SupplyChainSpec(nodes_info, **kwargs)
        elif kwargs:
            raise ValueError("keywords go into the SupplyChainSpec when a spec is given")
        n_envs = int(n_envs)
        if n_envs < 1:
            raise ValueError("n_envs must be >= 1")
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type != "cuda":
            raise ValueError("SupplyChainVecEnv runs on a GPU device (no CPU fallback)")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._dev_index = self.device.index
        if obs_dtype not in (torch.float32, torch.float64):
            raise ValueError("obs_dtype must be torch.float32 or torch.float64")
        self.spec = spec
        self.n_envs = n_envs
        self.auto_reset = bool(auto_reset)
        self.obs_dtype = obs_dtype
        P, NN = spec.P, len(spec.nodes)

        host_nodes = spec.node_table()
        # the chain as the spec resolved it, before scg_sc_prepare adds the chosen kernel's
        # inbox plan: part of the checkpoint fingerprint, which must not depend on the kernel
        self._nodes_digest = hashlib.sha256(bytes(host_nodes)).hexdigest()
        c = nat.ScConfig()
        c.n_nodes, c.n_products, c.n_retailers = NN, P, spec.n_retailers
        c.total_time_steps = spec.total_time_steps
        c.avg_leadtime, c.max_leadtime = spec.avg_leadtime, spec.max_leadtime
        c.stochastic_leadtimes = int(spec.stochastic_leadtimes)
        models = spec.demand_models
        c.demand_lo, c.demand_hi = models[0].lo, models[0].hi
        if any(m.kind != demand.UNIFORM or (m.lo, m.hi) != (models[0].lo, models[0].hi) for m in models):
            self._demand_tables(c, models, spec.total_time_steps)
        for k, v in spec.penalties.items():
            setattr(c, k, v)
        c.obs_f64 = int(obs_dtype == torch.float64)
        if kernel not in self._KERNELS:
            raise ValueError(f"kernel must be one of {sorted(self._KERNELS)}, got {kernel!r}")
        c.kernel = self._KERNELS[kernel]
        if spec.build_info and c.kernel == nat.SC_KERNEL_LEVEL:
            raise ValueError("build_info ledgers are kept by the lane, staged and node-parallel kernels "
                             "(kernel='lane', 'staged', 'nodes' or 'auto')")
        nat.check(nat.lib.scg_sc_prepare(ctypes.byref(c), host_nodes))
        self.kernel = {nat.SC_KERNEL_LEVEL: "level", nat.SC_KERNEL_STAGED: "staged",
                       nat.SC_KERNEL_NODES: "nodes"}.get(c.kernel, "lane")
        self._env_major = c.layout == nat.SC_LAYOUT_ENV_MAJOR
        if (c.n_actions, c.n_obs, c.n_leadtimes) != (spec.n_actions, spec.n_obs, spec.n_leadtimes):
            raise RuntimeError("host/library disagree on the chain's action/observation sizes")
        self._node_bytes = torch.frombuffer(bytearray(bytes(host_nodes)), dtype=torch.uint8).to(self.device)
        self._caller_tables = [demand_table is not None, leadtime_table is not None]
        c.nodes = self._node_bytes.data_ptr()
        if spec.stochastic_leadtimes:
            thr = nat.poisson_table(spec.avg_leadtime - 1)
            self._lt_thr = torch.tensor(np.asarray(thr, dtype=np.uint32).view(np.int32), device=self.device)
            c.leadtime_poisson = self._lt_thr.data_ptr()
            c.leadtime_poisson_len = len(thr)
        T, R = spec.total_time_steps, spec.n_retailers
        if demand_table is not None:
            if (demand_table.device != self.device or demand_table.dtype != torch.int32 or
                    tuple(demand_table.shape) != (n_envs, T + 1, R, P)):
                raise ValueError(f"demand_table must be int32 [{n_envs}, {T + 1}, {R}, {P}] on {self.device}")
            self._dem_tab = demand_table.contiguous()
            c.demand_table = self._dem_tab.data_ptr()
        if leadtime_table is not None:
            if not spec.stochastic_leadtimes:
                raise ValueError("leadtime_table needs stochastic_leadtimes=True")
            if (leadtime_table.device != self.device or leadtime_table.dtype != torch.int32 or
                    tuple(leadtime_table.shape) != (n_envs, T, spec.n_leadtimes)):
                raise ValueError(f"leadtime_table must be int32 [{n_envs}, {T}, {spec.n_leadtimes}] on {self.device}")
            lo, hi = int(leadtime_table.min()), int(leadtime_table.max())
            if lo < 1 or hi > spec.max_leadtime:  # the range the reference's draws have (:670-672)
                raise ValueError(f"leadtime_table values must lie in [1, max_leadtime={spec.max_leadtime}], "
                                 f"got [{lo}, {hi}]")
            self._lt_tab = leadtime_table.contiguous()
            c.leadtime_table = self._lt_tab.data_ptr()
        self._cfg = c
        self.n_actions, self.n_obs, self.heap_capacity = c.n_actions, c.n_obs, c.heap_capacity
        NP, H = NN * P, c.heap_capacity
        dev = self.device
        if self._env_major:  # [N][NP], [N][NP][H]: one env's chain is one contiguous block
            self._stock = torch.zeros((n_envs, NP), dtype=torch.float64, device=dev)
            self._heap_tk = torch.zeros((n_envs, NP, H), dtype=torch.int32, device=dev)
            self._heap_val = torch.zeros((n_envs, NP, H), dtype=torch.float64, device=dev)
            self._heap_size = torch.zeros((n_envs, NP), dtype=torch.int32, device=dev)
        else:  # env-fastest: lanes of a wave touching one slot read one contiguous row
            self._stock = torch.zeros((NP, n_envs), dtype=torch.float64, device=dev)
            self._heap_tk = torch.zeros((NP, H, n_envs), dtype=torch.int32, device=dev)
            self._heap_val = torch.zeros((NP, H, n_envs), dtype=torch.float64, device=dev)
            self._heap_size = torch.zeros((NP, n_envs), dtype=torch.int32, device=dev)
        self._err = torch.zeros(1, dtype=torch.int32, device=dev)
        self._inbox_tk = self._inbox_val = None
        if self.kernel == "staged":  # shipments in flight within a step [inbox_size][N]
            self._inbox_tk = torch.zeros((max(c.inbox_size, 1), n_envs), dtype=torch.uint8, device=dev)
            self._inbox_val = torch.zeros((max(c.inbox_size, 1), n_envs), dtype=torch.float64, device=dev)
        self._ret = torch.zeros(n_envs, dtype=torch.float64, device=dev) if track_returns else None
        self._final_ret = torch.zeros(n_envs, dtype=torch.float64, device=dev) if track_returns else None
        self._obs = torch.zeros((n_envs, c.n_obs), dtype=obs_dtype, device=dev)
        self._term_obs = torch.zeros((n_envs, c.n_obs), dtype=obs_dtype, device=dev)
        self._rew = torch.zeros(n_envs, dtype=torch.float64, device=dev)
        self._done_false = torch.zeros(n_envs, dtype=torch.bool, device=dev)
        self._done_true = torch.ones(n_envs, dtype=torch.bool, device=dev)
        s = nat.ScState()
        s.n_envs, s.env_offset, s.seed = n_envs, int(env_offset), _default_seed(seed, seed_group)
        s.episode, s.time_step = 0, -1
        s.stock, s.heap_tk, s.heap_val = self._stock.data_ptr(), self._heap_tk.data_ptr(), self._heap_val.data_ptr()
        s.heap_size, s.error_flags = self._heap_size.data_ptr(), self._err.data_ptr()
        if self._inbox_tk is not None:
            s.inbox_tk, s.inbox_val = self._inbox_tk.data_ptr(), self._inbox_val.data_ptr()
        s.episode_return = self._ret.data_ptr() if track_returns else None
        s.final_return = self._final_ret.data_ptr() if track_returns else None
        self.build_info = spec.build_info
        if self.build_info:  # [part][key][P][N], env fastest (include/scgpu.h)
            shape = (2, nat.SC_LEDGER_KEYS, P, n_envs)
            self._led = torch.zeros(shape, dtype=torch.float64, device=dev)
            self._led_k = torch.zeros(shape, dtype=torch.int32, device=dev)
            s.ledger, s.ledger_kind = self._led.data_ptr(), self._led_k.data_ptr()
            if self.auto_reset:
                self._fled = torch.zeros(shape, dtype=torch.float64, device=dev)
                self._fled_k = torch.zeros(shape, dtype=torch.int32, device=dev)
                s.final_ledger, s.final_ledger_kind = self._fled.data_ptr(), self._fled_k.data_ptr()
            if self.kernel == "nodes":  # each node's entry values of a step [NN * 2 * 8 * P][N]
                pshape = (NN * 2 * nat.SC_LEDGER_KEYS * P, n_envs)
                self._led_part = torch.zeros(pshape, dtype=torch.float64, device=dev)
                s.ledger_part = self._led_part.data_ptr()
            if not track_returns:
                raise ValueError("build_info needs track_returns (sc_episode['rewards'])")
        self._st = s
        self._cfg_ref, self._st_ref = ctypes.byref(self._cfg), ctypes.byref(self._st)
        self._done_flag = ctypes.c_int32(0)
        self._done_ref = ctypes.byref(self._done_flag)
        self._flags = nat.SCG_BG_AUTORESET if self.auto_reset else 0
        self._act_shape = (n_envs, c.n_actions)
        self._cfg_addr, self._st_addr = ctypes.addressof(self._cfg), ctypes.addressof(self._st)
        self._obs_ptr, self._rew_ptr, self._term_ptr = (self._obs.data_ptr(), self._rew.data_ptr(),
                                                        self._term_obs.data_ptr())
        self.single_action_space = spaces.Box(-1.0, 1.0, (c.n_actions,), np.float32)          # :625
        self.single_observation_space = spaces.Box(-1.0, 1.0, (c.n_obs,), np.float32)         # :626

    def _demand_tables(self, c, models, T):
        """Per-product demand models into the config; their tables onto the device."""
        self._dem_tabs = []

        def upload(a):
            t = torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).to(self.device)
            self._dem_tabs.append(t)
            return t.data_ptr()

        demand.fill_config(c, models, T, upload)

    def _stream(self):
        return nat.raw_stream(self._dev_index)

    def seed(self, seed=None, seed_group=None):
        """New Philox key and episode counter 0 (the reference re-creates its RandomState, :811-813);
        seed=None with `seed_group`: the group's rank 0 entropy (a collective)."""
        self._st.seed = _default_seed(seed, seed_group)
        self._st.episode = 0
        self._st.time_step = -1

    def reset(self):
        nat.check(nat.lib.scg_sc_reset(self._cfg_ref, self._st_ref, self._obs.data_ptr(), self._stream()))
        return self._obs

    def _actions(self, a):
        if not isinstance(a, torch.Tensor):
            a = torch.as_tensor(np.asarray(a, dtype=np.float32))
        if a.dtype != torch.float32 or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.float32)
        if a.shape != self._act_shape:
            if a.numel() != self._act_shape[0] * self._act_shape[1]:
                raise ValueError(f"actions must have shape {self._act_shape}, got {tuple(a.shape)}")
            a = a.reshape(self._act_shape)
        return a.contiguous()

    def step(self, actions):
        a = actions
        if not (type(a) is torch.Tensor and a.dtype is torch.float32 and a.is_cuda and
                a.get_device() == self._dev_index and a.shape == self._act_shape and a.is_contiguous()):
            a = self._actions(a)
        r = nat.fast.sc_step(self._cfg_addr, self._st_addr, a.data_ptr(), self._obs_ptr, self._rew_ptr,
                             self._term_ptr, self._flags, nat.raw_stream(self._dev_index))
        if r > 1:
            nat.check(r >> 1)
        if r & 1:
            self.check_errors()
            info = {"terminal_observation": self._term_obs}
            if self._final_ret is not None:
                info["episode_return"] = self._final_ret
            if self.build_info:
                info["sc_episode"] = self._ledger_views(self._led, self._ret if self.auto_reset else self._final_ret)
                if self.auto_reset:
                    info["terminal_sc_episode"] = self._ledger_views(self._fled, self._final_ret)
            return self._obs, self._rew, self._done_true, info
        if self.build_info:
            return self._obs, self._rew, self._done_false, {"sc_episode": self._ledger_views(self._led, self._ret)}
        return self._obs, self._rew, self._done_false, {}

    def _ledger_views(self, led, rewards):
        P, names = self.spec.P, nat.SC_LEDGER_NAMES
        return {"rewards": rewards,
                "costs": {k: led[0, j].permute(1, 0) for j, k in enumerate(names)},
                "units": {k: led[1, j].permute(1, 0) for j, k in enumerate(names)}}

    def ledger_kinds(self, final=False):
        """NumPy type codes [2, 8, P, N] of the ledger entries (0 int, 1 float, 2 float32,
        3 float64, 4 int64)."""
        return self._fled_k if final else self._led_k

    def sc_episode(self, env, final=False):
        """info['sc_episode'] of one env as the reference builds it (:684-695): Python /
        NumPy scalars of the reference's types, lists per product."""
        if not self.build_info:
            raise ValueError("the env was built with build_info=False")
        led, kinds, ret = (self._fled, self._fled_k, self._final_ret) if final else (self._led, self._led_k, self._ret)
        v = led[..., env].cpu().numpy()
        k = kinds[..., env].cpu().numpy()
        out = {"rewards": np.float64(ret[env].item())}
        for part, name in ((0, "costs"), (1, "units")):
            out[name] = {key: [_SC_TYPES[int(k[part, j, p])](v[part, j, p]) for p in range(self.spec.P)]
                         for j, key in enumerate(nat.SC_LEDGER_NAMES)}
        return out

    @property
    def kernel_symbol(self):
        """The step kernel scg_sc_step launches for this batch, as rocprofv3 names it (the
        lane kernel keeps every heap in LDS when a block's share fits 64 KiB)."""
        c = self._cfg
        d = c.max_dests
        maxd = 2 if d <= 2 else 4 if d <= 4 else 8 if d <= 8 else 16 if d <= 16 else 32
        if self.kernel == "level":
            return f"scg::sc_level_kernel<{maxd}, {'true' if c.level_staged else 'false'}>"
        if self.kernel == "staged":
            return f"scg::sc_step_staged_kernel<{maxd}, {'true' if self.build_info else 'false'}>"
        if self.kernel == "nodes":
            return (f"scg::sc_step_nodes_kernel<{maxd}, {'true' if c.obs_f64 else 'false'}, "
                    f"{'true' if self.build_info else 'false'}>")
        lds = 64 * len(self.spec.nodes) * self.spec.P * (12 * c.heap_capacity + 4)
        if lds > 64 * 1024:
            return f"scg::sc_step_kernel<{maxd}>"
        # envs per block as scg_supplychain.hip sc_lds_epb picks them: half-full waves when
        # full ones would give a SIMD fewer than two
        cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        epb = 32 if self.n_envs < cus * 4 * 2 * 64 else 64
        return f"scg::sc_step_lds_kernel<{maxd}, {epb}>"

    def check_errors(self):
        """Raise if any env's in-transit heap overflowed its capacity (never expected: the
        capacity is the chain's provable bound, scg_sc_prepare)."""
        if int(self._err.item()):
            raise RuntimeError("in-transit heap capacity exceeded; results are invalid")

    # checkpoint / resume (gym_supplychain_amd/checkpoint.py) ------------------
    # kernel-choice outputs of scg_sc_prepare: a checkpoint moves between kernels (the level
    # kernel alone fills the level schedule)
    _CKPT_SKIP = ("kernel", "layout", "group", "level_staged", "inbox_size", "n_levels", "level_start")

    def _ckpt_buffers(self):
        """Every device buffer that carries state from one step to the next, heaps and stocks
        viewed env-major ([N, NP], [N, NP, H]) whatever the kernel's layout, so a checkpoint
        restores into any kernel; the staged kernel's inbox and the node-parallel kernel's
        ledger slots live within one step and are not state."""
        led = self.build_info
        fled = led and self.auto_reset
        if self._env_major:
            stock, tk, val, size = self._stock, self._heap_tk, self._heap_val, self._heap_size
        else:
            stock, size = self._stock.t(), self._heap_size.t()
            tk, val = self._heap_tk.permute(2, 0, 1), self._heap_val.permute(2, 0, 1)
        return {"stock": stock, "heap_tk": tk, "heap_val": val, "heap_size": size, "error_flags": self._err,
                "episode_return": self._ret, "final_return": self._final_ret, "obs": self._obs,
                "terminal_observation": self._term_obs, "reward": self._rew,
                "ledger": self._led if led else None, "ledger_kind": self._led_k if led else None,
                "final_ledger": self._fled if fled else None, "final_ledger_kind": self._fled_k if fled else None}

    def _ckpt_fingerprint(self):
        return ckpt.config_fingerprint(self._cfg, skip=self._CKPT_SKIP) + [
            ["n_envs", self.n_envs], ["env_offset", int(self._st.env_offset)], ["auto_reset", int(self.auto_reset)],
            ["nodes_sha256", self._nodes_digest], ["caller_tables", list(self._caller_tables)]]

    def state_dict(self):
        """Checkpoint of every env: stocks, in-transit heaps (CPython storage order), ledgers,
        returns and the last outputs (cloned on the current stream, after every step already
        enqueued) with the Philox key, episode and time step. load_state_dict() on an env of
        the same chain and batch, any kernel, resumes bit for bit. Caller demand / lead-time
        tables are inputs, not state: pass the same ones to the new env."""
        return ckpt.snapshot(type(self).__name__, self._ckpt_fingerprint(),
                             {"seed": self._st.seed, "episode": self._st.episode, "time_step": self._st.time_step},
                             self._ckpt_buffers())

    def load_state_dict(self, state):
        """Restore a state_dict() of an env of the same chain and batch (ValueError
        otherwise); the copies are enqueued on the current stream."""
        bufs = self._ckpt_buffers()
        ckpt.check(state, type(self).__name__, self._ckpt_fingerprint(), bufs)
        cnt = ckpt.restore(state, bufs)
        self._st.seed, self._st.episode, self._st.time_step = cnt["seed"], cnt["episode"], cnt["time_step"]

    def draw_tables(self, episode=None):
        """(demand int32 [N, T+1, R, P], lead times int32 [N, T, n_lt] or None) for an episode."""
        sp = self.spec
        ep = self._st.episode if episode is None else int(episode)
        dem = torch.empty((self.n_envs, sp.total_time_steps + 1, sp.n_retailers, sp.P), dtype=torch.int32,
                          device=self.device)
        lts = None
        if sp.stochastic_leadtimes:
            lts = torch.empty((self.n_envs, sp.total_time_steps, sp.n_leadtimes), dtype=torch.int32,
                              device=self.device)
        nat.check(nat.lib.scg_sc_draw_tables(self._cfg_ref, self._st_ref, ep, dem.data_ptr(),
                                             lts.data_ptr() if lts is not None else None, self._stream()))
        return dem, lts

    # state views ----------------------------------------------------------------------
    @property
    def time_step(self):
        return self._st.time_step

    @property
    def episode(self):
        return self._st.episode

    @property
    def env_offset(self):
        return self._st.env_offset

    @property
    def stock(self):
        """[N, nodes, P] float64 view of every node's stock."""
        if self._env_major:
            return self._stock.view(self.n_envs, len(self.spec.nodes), self.spec.P)
        return self._stock.view(len(self.spec.nodes), self.spec.P, self.n_envs).permute(2, 0, 1)

    @property
    def episode_return(self):
        return self._ret

    @property
    def final_return(self):
        return self._final_ret

    def heaps(self, env):
        """In-transit heaps of one env as the reference's shipments_by_prod lists
        [node][product] -> [(time, amount), ...] in storage order."""
        P = self.spec.P
        if self._env_major:
            tk, val, size = (self._heap_tk[env].cpu().numpy(), self._heap_val[env].cpu().numpy(),
                             self._heap_size[env].cpu().numpy())
        else:
            tk = self._heap_tk[:, :, env].cpu().numpy()
            val = self._heap_val[:, :, env].cpu().numpy()
            size = self._heap_size[:, env].cpu().numpy()
        out = []
        for i in range(len(self.spec.nodes)):
            out.append([[(int(tk[i * P + p, j]) >> 3, float(val[i * P + p, j])) for j in range(size[i * P + p])]
                        for p in range(P)])
        return out

    def close(self):
        pass


class SC_NodeView:
    """Read-only view of one chain node of a drop-in env, with the attributes the
    reference's SC_Node exposes and its tests read (supplychain_env.py:120-176): `stock`
    (float64 array, :228), `shipments_by_prod` (per product, the in-transit heap as a list
    of (time, amount) tuples in heapq storage order, :175, :398-400), capacities and costs.
    Each access reads the device state back."""

    def __init__(self, env, index):
        self._env, self._i = env, index
        nd = env._vec.spec.nodes[index]
        self.label = nd["name"]
        self.num_products = env._vec.spec.P
        self.last_level = nd["last_level"]
        self.stock_capacities = list(nd["stock_capacity"])
        self.stock_cost = list(nd["stock_cost"])
        self.max_ship = list(nd["max_ship"])
        self.processing_capacity = nd["processing_capacity"]
        self.num_supply_actions, self.num_ship_actions = nd["n_supply"], nd["n_ship"]

    @property
    def stock(self):
        return self._env._vec.stock[0, self._i].cpu().numpy().copy()

    @property
    def shipments_by_prod(self):
        return self._env._vec.heaps(0)[self._i]

    def num_expected_actions(self):
        return self.num_supply_actions + self.num_ship_actions

    def is_last_level(self):
        return self.last_level

    def __repr__(self):
        return f"{self.label} ({self.shipments_by_prod}) [{np.round(self.stock, 1)}]"


class _ScStepServer:
    """The drop-in SupplyChainEnv's step server (include/scgpu.h scg_sc_server_*): one
    resident block of the node-parallel kernel's shape on a non-blocking, high-priority stream
    of its own polls a host-mapped mailbox and runs each posted step on the env's state (the
    batch kernel's tile code), writing observation and reward to the env's host-mapped block.
    It exits when stopped (reset(), close(), another server of the device becoming resident,
    interpreter exit) or by itself after IDLE_US without a request; step() launches it again
    when needed. The mailbox is freed only after the block has been stopped."""

    IDLE_US = 20000

    def __init__(self, vec, act_dev, act_host, obs_dev, rew_dev):
        stream, self.priority = resident.server_stream(vec.device)
        self._dev_index = vec._dev_index
        self._device = vec.device
        self._box = box = nat.MappedBuffer(ctypes.sizeof(nat.ScServerBox))
        self.box = nat.ScServerBox.from_address(box.host)
        self.sv = nat.ScServer(box.host, box.dev, stream, act_dev, act_host, obs_dev, rew_dev, self.IDLE_US, 0)
        self._args = (vec._cfg_addr, vec._st_addr, ctypes.addressof(self.sv))
        self._fast = nat.fast.sc_server_step
        self._closed = False
        _SC_SERVERS.add(self)

    @property
    def launches(self):
        return int(self.sv.launches)

    def step(self):
        resident.claim(self._dev_index, self)
        return self._fast(*self._args)

    def stop(self):
        if not self._closed:
            with torch.cuda.device(self._device):
                nat.check(nat.lib.scg_sc_server_stop(ctypes.byref(self.sv)))

    def close(self):
        if self._closed:
            return
        self.stop()  # raises if the block cannot be stopped: then the mailbox stays allocated
        self._closed = True
        resident.release(self._dev_index, self)
        resident.destroy_stream(self.sv.stream)
        self._box = None
        _SC_SERVERS.discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter teardown
            pass


_SC_SERVERS = weakref.WeakSet()


@atexit.register
def _stop_sc_servers():  # no server block outlives the interpreter (nor its mailbox)
    for sv in list(_SC_SERVERS):
        sv.close()


class SupplyChainEnv(spaces.Env):
    """Drop-in for gym_supplychain.envs.SupplyChainEnv (:478-813), one env on the GPU.

    Same constructor keywords; reset() -> float64 obs in [-1, 1]; step(action) ->
    (obs, np.float64 reward, done, info); seed(seed) re-creates the RandomState and seeds
    action_space with 0 (:811-813). info is {} or, with build_info, {'sc_episode':
    ledgers} (one dict per episode, updated in place each step).

    host_rng=True (default): each reset() draws the episode's demand and lead times from
    the env's RandomState exactly as the reference does (:564, :644-672; envs/host_rng.py)
    and uploads them, so seeded episodes are the reference's, draw for draw.
    host_rng=False: Philox draws on the device from `seed` (module docstring).
    The reference's attributes `customer_demands`, `leadtimes`, `nodes` (SC_NodeView),
    `count_leadtimes_per_timestep` and `rand_generator` are kept.
    kernel=None (default): the node-parallel kernel when the chain qualifies (one env is a
    latency path: every node on its own wave), else the vec env's "auto" choice; or name one
    ("lane", "staged", "level", "nodes", "auto"). On the node-parallel kernel without
    build_info each step is posted to a resident block (the step server, include/scgpu.h
    scg_sc_server_*) rather than launched; the block exits 20 ms after the last step, so a
    device-wide torch.cuda.synchronize() right after a step waits up to that long.
    SCG_SC_SERVER=0 launches the kernel per step instead.
    """

    def __init__(self, nodes_info, num_products=1, unmet_demand_cost=1000, exceeded_stock_capacity_cost=1000,
                 exceeded_process_capacity_cost=1000, exceeded_ship_capacity_cost=1000,
                 demand_config_by_product=False, demand_range=(10, 20), demand_std=None, demand_sen_peaks=None,
                 avg_demand_range=None, processing_ratio=3, stochastic_leadtimes=False, avg_leadtime=2,
                 max_leadtime=2, total_time_steps=360, seed=None, build_info=False, demand_perturb_norm=False,
                 device=None, host_rng=True, kernel=None):
        dkw = dict(demand_config_by_product=demand_config_by_product, demand_range=demand_range,
                   demand_std=demand_std, demand_sen_peaks=demand_sen_peaks, avg_demand_range=avg_demand_range,
                   demand_perturb_norm=demand_perturb_norm)
        spec = SupplyChainSpec(nodes_info, num_products=num_products, unmet_demand_cost=unmet_demand_cost,
                               exceeded_stock_capacity_cost=exceeded_stock_capacity_cost,
                               exceeded_process_capacity_cost=exceeded_process_capacity_cost,
                               exceeded_ship_capacity_cost=exceeded_ship_capacity_cost,
                               processing_ratio=processing_ratio,
                               stochastic_leadtimes=stochastic_leadtimes, avg_leadtime=avg_leadtime,
                               max_leadtime=max_leadtime, total_time_steps=total_time_steps, seed=seed,
                               build_info=build_info, **dkw)
        T, R, P = spec.total_time_steps, spec.n_retailers, spec.P
        self._host = None
        vec_kw = {}
        if host_rng:
            from .host_rng import HostEpisodeDraws
            self._host = HostEpisodeDraws(dkw, R, P, T, spec.n_leadtimes, spec.stochastic_leadtimes,
                                          spec.avg_leadtime, spec.max_leadtime, seed)
            dev = torch.device(device) if device is not None else torch.device("cuda")
            vec_kw["demand_table"] = torch.zeros((1, T + 1, R, P), dtype=torch.int32, device=dev)
            if spec.stochastic_leadtimes:
                vec_kw["leadtime_table"] = torch.ones((1, T, spec.n_leadtimes), dtype=torch.int32, device=dev)
        # One env is a latency path, not an occupancy one: the node-parallel kernel (every node
        # of the env on its own wave) whenever the chain qualifies, which the "auto" choice, made
        # for batches, skips when two blocks of it would not share a CU (sc-2perstage, float64
        # observations: 26.9 against 58.3 us per step() for the lane kernel,
        # profiles/r05zz_sc_facade_kernels.log); otherwise the auto choice.
        self._vec = None
        if kernel is None:
            try:
                self._vec = SupplyChainVecEnv(1, spec=spec, seed=seed, device=device, auto_reset=False,
                                              obs_dtype=torch.float64, kernel="nodes", **vec_kw)
            except ValueError:  # the chain does not qualify (scg_sc_prepare)
                self._vec = None
        if self._vec is None:
            self._vec = SupplyChainVecEnv(1, spec=spec, seed=seed, device=device, auto_reset=False,
                                          obs_dtype=torch.float64, kernel=kernel or "auto", **vec_kw)
        self.num_products = spec.P
        self.total_time_steps = spec.total_time_steps
        self.stochastic_leadtimes = spec.stochastic_leadtimes
        self.avg_leadtime, self.max_leadtime = spec.avg_leadtime, spec.max_leadtime
        self.demand_range = spec.demand_range
        self.demand_config_by_product = spec.demand_config_by_product
        if spec.stochastic_leadtimes:
            self.count_leadtimes_per_timestep = spec.n_leadtimes                       # :601-605
        self.action_space = spaces.Box(-1.0, 1.0, (spec.n_actions,), np.float32)   # :625
        self.observation_space = spaces.Box(-1.0, 1.0, (spec.n_obs,), np.float32)  # :626
        self.nodes = [SC_NodeView(self, i) for i in range(len(spec.nodes))]
        self.last_level_nodes = [nd for nd in self.nodes if nd.last_level]
        self.current_state = None
        self.current_reward = 0
        self.customer_demands = None
        self.leadtimes = None
        # the step's action, observation and reward in one host-mapped block: a step is one
        # launch and one stream synchronisation, no copies (profiles/r05*_facade_latency.log)
        A, O = spec.n_actions, spec.n_obs
        ra = (4 * A + 15) // 16 * 16
        self._io = io = nat.MappedBuffer(ra + 8 * O + 8)
        self._act_np = io.view(np.float32, 0, A).reshape(1, A)
        self._act_row, self._n_act = self._act_np[0], A
        self._obs_np = io.view(np.float64, ra, O)
        self._rew_np = io.view(np.float64, ra + 8 * O, 1)
        self._io_ptrs = (io.dev, io.dev + ra, io.dev + ra + 8 * O)
        self._sync = nat.stream_synchronize_fn()
        self.build_info = spec.build_info
        self.est_episode = None
        # On the node-parallel kernel (float64 observations, no ledgers) the step runs on a
        # resident block polling a mailbox (scg_sc_server_*): no launch and no stream
        # synchronisation per step. SCG_SC_SERVER=0: one launch plus one synchronisation.
        self._server = None
        if os.environ.get("SCG_SC_SERVER", "1") != "0" and self._vec.kernel == "nodes" and not self.build_info:
            act, obs, rew = self._io_ptrs
            self._server = _ScStepServer(self._vec, act, io.host, obs, rew)

    @property
    def time_step(self):
        return self._vec.time_step

    @property
    def rand_generator(self):
        """The reset-time RandomState (host_rng mode), as the reference's attribute (:564)."""
        return self._host.rng if self._host is not None else None

    def seed(self, seed=None):
        """:811-813 — a new RandomState(seed) for the episode draws (host_rng; the Philox key
        otherwise), and action_space.seed(0)."""
        if self._host is not None:
            self._host.seed(seed)
        else:
            self._vec.seed(seed)
        self.action_space.seed(0)

    def _upload_episode_tables(self):
        """Draw this episode's tables on the host (reference order) and copy them to the
        device tables the kernels read; synchronous copies from pageable memory, so the
        host buffers may be reused at once."""
        dem, table, lts = self._host.draw()
        self.customer_demands = dem
        self._vec._dem_tab.copy_(torch.from_numpy(table).unsqueeze(0))
        if lts is not None:
            self.leadtimes = lts
            self._vec._lt_tab.copy_(torch.from_numpy(lts.astype(np.int32)).unsqueeze(0))

    def reset(self):
        if self._host is not None:
            self._upload_episode_tables()
        obs = self._vec.reset()
        if self._host is None:  # Philox draws of this episode, read back for the attributes
            dem, lts = self._vec.draw_tables()
            self.customer_demands = dem[0].cpu().numpy().astype(np.int64)
            self.leadtimes = None if lts is None else lts[0].cpu().numpy().astype(np.int64)
        self.current_reward = 0
        self.episode_rewards = 0
        if self.build_info:  # a new ledger dict per episode, mutated by every step (:677-678, :796)
            self.est_episode = self._vec.sc_episode(0)
            self.est_episode["rewards"] = 0
        self.current_state = obs[0].cpu().numpy().copy()
        return self.current_state

    def step(self, action):
        # (the per-call Python here is part of the step's latency: a float32 vector, the
        # usual case, goes straight into the host-mapped action row)
        a = action
        if type(a) is not np.ndarray or a.dtype != np.float32 or a.ndim != 1:
            a = np.asarray(a, dtype=np.float32).reshape(-1)
        n = self._n_act
        if a.size != n:
            if a.size < n:  # the reference's per-node slices run past the end (:716-717 -> act)
                raise IndexError(f"action has {a.size} values, the chain needs {n}")
            a = a[:n]  # like the reference, values beyond the chain's actions are unused
        self._act_row[:] = a
        v = self._vec
        srv = self._server
        if srv is not None:
            r = srv.step()  # returns once the block has written obs and reward
            if r > 1:
                nat.check(r >> 1)
        else:
            stream = nat.raw_stream(v._dev_index)
            act, obs, rew = self._io_ptrs
            r = nat.fast.sc_step(v._cfg_addr, v._st_addr, act, obs, rew, v._term_ptr, v._flags, stream)
            if r > 1:
                nat.check(r >> 1)
            rc = self._sync(stream)
            if rc:
                raise RuntimeError(f"hipStreamSynchronize failed ({rc})")
        self.current_state = obs = self._obs_np.copy()
        self.current_reward = rew = self._rew_np[0]  # an np.float64 (:734)
        self.episode_rewards += rew
        done = v._st.time_step == self.total_time_steps
        if done:
            v.check_errors()
        if self.build_info:
            self.est_episode.update(v.sc_episode(0))
            return obs, rew, done, {"sc_episode": self.est_episode}
        return obs, rew, done, {}

    @property
    def stock(self):
        return self._vec.stock[0].cpu().numpy()

    def shipments(self):
        return self._vec.heaps(0)

    def render(self, mode='human'):
        print('TIMESTEP:', self.time_step)
        st = self.stock
        for i, name in enumerate(self._vec.spec.node_names):
            print(f'{name} {self.shipments()[i]} [{np.round(st[i], 1)}]')
        print('Current state :', self.current_state)
        print('Current reward:', round(float(self.current_reward), 3))

    def close(self):
        server = getattr(self, "_server", None)
        if server is not None:
            server.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter teardown
            pass
