"""MIT Beer Game on MI355X: batched ``BeerGameVecEnv`` and the drop-in ``BeerGameEnv``.

Mirrors gym_supplychain.envs.BeerGameEnv (gym_supplychain/envs/beergame_env.py,
reference snapshot 2024-08-07): same env_init_info keys and defaults (:16-43), same
reset()/step() results (:66-156), same exceptions for the same misuse. The dynamics run
in HIP kernels (gym-supplychain_amd/csrc/scg_beergame.hip) through the C ABI of
include/scgpu.h; this module only owns device buffers and marshals arguments.

Differences from the reference, all documented in DESIGN.md:
  * state is int32 (the reference's int64 values are reproduced exactly while they fit);
  * actions are integers — a float action is truncated toward zero on input;
  * BeerGameVecEnv adds per-env demand (a device table, or Poisson draws made on device
    with Philox4x32-10) and auto-reset; the reference has one fixed demand list (F2).
"""
import atexit
import ctypes
import numbers
import os
import weakref

import numpy as np
import torch

from .. import _native as nat
from .. import checkpoint as ckpt
from .. import spaces
from . import resident
from ..distributed import entropy_seed

# beergame_env.py:16-23
STD_LEVELS = 4
STD_DEMAND = [4] * 4 + [8] * 31
STD_INVENTORY = 12
STD_SHIP_DELAY = 2
STD_SHIP_VALUE = 4
STD_ORDERS_VALUE = 4
STD_INV_COST = 1
STD_BACKLOG_COST = 2

_I32 = (-(2 ** 31), 2 ** 31 - 1)
# sampled actions of the vec envs' Box stay int32-exact over an episode (|a| <= 2^15)
ACTION_BOUND = 2 ** 15


_entropy_seed = entropy_seed  # seed=None: this process's entropy unless a seed_group is given


def _int32(name, v):
    if isinstance(v, (bool, np.bool_)) or not isinstance(v, (numbers.Integral, np.integer)):
        # the reference's ledgers are int arrays: a float cost fails at its first step (:131)
        raise TypeError(f"{name} must be an integer, got {type(v).__name__}")
    v = int(v)
    if not _I32[0] <= v <= _I32[1]:
        raise ValueError(f"{name}={v} does not fit int32")
    return v


def _int32_list(name, seq):
    arr = np.asarray(seq)
    if arr.dtype.kind == "f":
        arr = arr.astype(np.int64)  # np.asarray(..., dtype=int) truncation (:33, :35)
    arr = arr.astype(np.int64).reshape(-1)
    if arr.size and (arr.min() < _I32[0] or arr.max() > _I32[1]):
        raise ValueError(f"{name} does not fit int32")
    return arr.astype(np.int32)


class BeerGameConfig:
    """env_init_info resolved as BeerGameEnv.__init__ does (beergame_env.py:11-58)."""

    def __init__(self, env_init_info=None, horizon=None):
        info = dict(env_init_info or {})
        self.levels = _int32("levels", info.get("levels", STD_LEVELS))
        if not 1 <= self.levels <= nat.BG_MAX_LEVELS:
            raise ValueError(f"levels={self.levels} outside 1..{nat.BG_MAX_LEVELS}")
        self.inv_cost = _int32("inv_cost", info.get("inv_cost", STD_INV_COST))
        self.backlog_cost = _int32("backlog_cost", info.get("backlog_cost", STD_BACKLOG_COST))
        self.customer_demand = _int32_list("customer_demand", info.get("customer_demand", STD_DEMAND))
        # T = len(customer_demand) (:37); a per-env demand source may set its own horizon
        self.max_weeks = int(horizon) if horizon is not None else int(self.customer_demand.size)
        if not 1 <= self.max_weeks <= nat.BG_MAX_WEEKS:
            raise ValueError(f"episode length {self.max_weeks} outside 1..{nat.BG_MAX_WEEKS}")
        inv0 = info.get("initial_inventory", STD_INVENTORY + np.zeros(STD_LEVELS))
        self.initial_inventory = _int32_list("initial_inventory", inv0)
        if self.initial_inventory.size != self.levels:
            # the reference fails later with a broadcast error; fail at construction
            raise ValueError(f"initial_inventory has {self.initial_inventory.size} entries, levels={self.levels}")
        # :39 — index 0 is the initial pipeline delay, always 2, then one delay per week
        user_delays = info.get("shipment_delays", [STD_SHIP_DELAY] * self.max_weeks)
        if isinstance(user_delays, np.ndarray):
            user_delays = user_delays.tolist()
        self.shipment_delays = _int32_list("shipment_delays", [STD_SHIP_DELAY] + list(user_delays))
        if self.shipment_delays.size < self.max_weeks + 1:
            # the reference's table sizing reads shipment_delays[0..T] (:47-48)
            raise IndexError(f"shipment_delays needs {self.max_weeks} entries, got {self.shipment_delays.size - 1}")
        self.shipment_delays = self.shipment_delays[: self.max_weeks + 1].copy()
        if self.shipment_delays.min() < 0 or self.shipment_delays.max() > nat.BG_MAX_DELAY:
            raise ValueError(f"shipment delays must be within 0..{nat.BG_MAX_DELAY}")
        self.initial_shipment_value = _int32("initial_shipment_value",
                                             info.get("initial_shipment_value", STD_SHIP_VALUE))
        self.initial_orders_value = _int32("initial_orders_value", info.get("initial_orders_value", STD_ORDERS_VALUE))


class BeerGameVecEnv:
    """N lock-step Beer Game envs on one GPU, state resident in HBM.

    reset() -> obs int32 [N, L]
    step(actions int32 [N, L]) -> (obs [N, L], reward int32 [N], done bool [N], info)

    Returned tensors are views of this env's output buffers, overwritten by the next
    call (clone() to keep them). With auto_reset (default) the step that reaches the
    terminal week resets every env in the same kernel: obs is then the reset
    observation and info holds 'terminal_observation' and 'episode_return'.

    demand: "fixed" — env_init_info['customer_demand'] for every env (reference);
            "poisson" — Poisson(poisson_lambda) per (env, episode, week), Philox4x32-10
                        keyed by `seed`, counter (env_offset + n, episode, week, 0);
            a device tensor int32 [T, N] — caller-supplied per-env demand.
    env_offset: global id of env 0 — shards on several GPUs draw the same per-env
            demand as one big batch would (multi-GPU invariant).
    state_slab: hold the state in one slab (scg_bg_slab_layout) so step() runs the slab
            kernel (default; needs N * L % 4 == 0, else separate buffers and the general
            kernel). Both give identical results.
    full_table: keep the reference's whole absolute-week shipment table (beergame_env.py:46-50)
            instead of the ring of max delay + 1 weeks (`shipment_table()`), any row count (past
            127 rows the state is not one slab: the general step kernel runs).
    Values the reference keeps in int64 are int32 here; a step whose int64 result leaves
    int32 sets a sticky device flag, raised as OverflowError by check_errors() and, one
    episode late (so the step loop never stalls), by the terminal step.
    """

    def __init__(self, n_envs, env_init_info=None, demand="fixed", poisson_lambda=8.0, seed=0, device=None,
                 env_offset=0, auto_reset=True, track_costs=True, track_history=False, track_returns=True,
                 horizon=None, config=None, variant_fields=None, state_slab=True, full_table=False):
        n_envs = int(n_envs)
        if n_envs < 1:
            raise ValueError("n_envs must be >= 1")
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type != "cuda":
            raise ValueError("BeerGameVecEnv runs on a GPU device (no CPU fallback)")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._dev_index = self.device.index
        table = None
        demand_range = (0, 0)
        if isinstance(demand, torch.Tensor):
            table = demand
            horizon = table.shape[0]
            mode = nat.SCG_DEMAND_TABLE
        elif isinstance(demand, tuple) and len(demand) == 3 and demand[0] == "uniform":
            mode, demand_range = nat.SCG_DEMAND_UNIFORM, (int(demand[1]), int(demand[2]))
        elif demand == "fixed":
            mode = nat.SCG_DEMAND_FIXED
        elif demand == "poisson":
            mode = nat.SCG_DEMAND_POISSON
        else:
            raise ValueError(f"demand must be 'fixed', 'poisson', ('uniform', lo, hi) or a device tensor, "
                             f"got {demand!r}")
        cfg = config if config is not None else BeerGameConfig(env_init_info, horizon=horizon)
        if mode == nat.SCG_DEMAND_FIXED and cfg.customer_demand.size < cfg.max_weeks:
            raise ValueError("customer_demand shorter than the horizon")
        self.config = cfg
        self.n_envs = n_envs
        self.levels = L = cfg.levels
        self.max_weeks = T = cfg.max_weeks
        self.auto_reset = bool(auto_reset)
        self.demand_mode = mode

        # host-side arrays the C ABI reads (kept alive on self)
        self._delays = (ctypes.c_int32 * (T + 1))(*cfg.shipment_delays.tolist())
        self._demand = (ctypes.c_int32 * max(T, 1))(*cfg.customer_demand[:T].tolist()) \
            if mode == nat.SCG_DEMAND_FIXED else None
        self._plan = (ctypes.c_int32 * (T + 1))()

        c = nat.BgConfig()
        c.levels, c.max_weeks = L, T
        c.inv_cost, c.backlog_cost = cfg.inv_cost, cfg.backlog_cost
        c.initial_shipment_value = cfg.initial_shipment_value
        c.initial_orders_value = cfg.initial_orders_value
        for i, v in enumerate(cfg.initial_inventory.tolist()):
            c.initial_inventory[i] = v
        c.demand_mode = mode
        c.demand_lo, c.demand_hi = demand_range
        c.full_table = int(bool(full_table))
        for k, v in (variant_fields or {}).items():
            setattr(c, k, v)
        c.shipment_delays = ctypes.cast(self._delays, ctypes.c_void_p)
        c.customer_demand = ctypes.cast(self._demand, ctypes.c_void_p) if self._demand is not None else None
        c.plan = ctypes.cast(self._plan, ctypes.c_void_p)
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        if mode == nat.SCG_DEMAND_TABLE:
            if table.device != dev or table.dtype != torch.int32 or tuple(table.shape) != (T, n_envs):
                raise ValueError(f"demand table must be int32 [{T}, {n_envs}] on {dev}")
            self._table = table.contiguous()
            c.demand_table = self._table.data_ptr()
        if mode == nat.SCG_DEMAND_POISSON:
            thr = nat.poisson_table(poisson_lambda)
            self.poisson_lambda = float(poisson_lambda)
            self._thresholds = torch.tensor(np.asarray(thr, dtype=np.uint32).view(np.int32), **i32)
            c.poisson_thresholds = self._thresholds.data_ptr()
            c.poisson_len = len(thr)
        nat.check(nat.lib.scg_bg_prepare(ctypes.byref(c)))
        self._cfg = c
        self.ring_slots = R = c.ring_slots

        # device state, env-major [N][L] int32 (DESIGN.md "Layout in HBM"): one slab holding
        # every row at the offsets scg_bg_slab_layout gives (the slab step kernel addresses
        # them all from one base), or separate tensors when N * L is not a multiple of 4
        v2 = c.variant == 2
        off = (ctypes.c_int64 * nat.SLAB_FIELDS)()
        self._slab = None
        if state_slab and nat.lib.scg_bg_slab_layout(ctypes.byref(c), n_envs, int(bool(track_history)), off) == 0:
            self._slab = torch.zeros(off[nat.SLAB_TOTAL], **i32)

            def rows(field, k=1):
                return self._slab[off[field]: off[field] + k * n_envs * L].view(*((k,) if k > 1 else ()), n_envs, L)

            def i64(field):
                return self._slab[off[field]: off[field] + 2 * n_envs].view(torch.int64)

            self._err = self._slab[off[nat.SLAB_ERROR]: off[nat.SLAB_ERROR] + 1]
            self._inv, self._bk, self._op = rows(nat.SLAB_INVENTORY), rows(nat.SLAB_BACKLOG), rows(nat.SLAB_ORDERS)
            self._ring = rows(nat.SLAB_RING, R) if R > 1 else rows(nat.SLAB_RING).unsqueeze(0)
            self._inv_costs = rows(nat.SLAB_INV_COSTS) if track_costs else None
            self._bk_costs = rows(nat.SLAB_BACKLOG_COSTS) if track_costs else None
            self._hist = rows(nat.SLAB_HISTORY, T + 1) if track_history else None
            self._ret = i64(nat.SLAB_EPISODE_RETURN) if track_returns else None
            self._final_ret = i64(nat.SLAB_FINAL_RETURN) if track_returns else None
            self._term_obs = rows(nat.SLAB_TERMINAL_OBS)
        else:
            self._err = torch.zeros(1, **i32)
            self._inv = torch.zeros((n_envs, L), **i32)
            self._bk = torch.zeros((n_envs, L), **i32)
            self._op = torch.zeros((n_envs, L), **i32)
            self._ring = torch.zeros((R, n_envs, L), **i32)
            self._inv_costs = torch.zeros((n_envs, L), **i32) if track_costs else None
            self._bk_costs = torch.zeros((n_envs, L), **i32) if track_costs else None
            self._hist = torch.zeros((T + 1, n_envs, L), **i32) if track_history else None
            self._ret = torch.zeros(n_envs, dtype=torch.int64, device=dev) if track_returns else None
            self._final_ret = torch.zeros(n_envs, dtype=torch.int64, device=dev) if track_returns else None
            self._term_obs = torch.zeros((n_envs, L), **i32)
        self._pen_costs = torch.zeros((n_envs, L), **i32) if (track_costs and v2) else None
        # outputs: obs and reward share one allocation so N=1 callers copy back once (and the
        # slab kernel writes both from one preloaded base)
        self._out = torch.zeros(n_envs * L + n_envs, **i32)
        self._obs = self._out[: n_envs * L].view(n_envs, L)
        self._rew = self._out[n_envs * L:]
        self._done_false = torch.zeros(n_envs, dtype=torch.bool, device=dev)
        self._done_true = torch.ones(n_envs, dtype=torch.bool, device=dev)
        # int32 overflow word: each terminal-week launch copies it to host-mapped memory, and
        # the host reads that copy at terminal steps (check_errors() reads the device word),
        # so the check never stalls the step pipeline
        self._err_word = nat.MappedWord()

        s = nat.BgState()
        s.n_envs, s.env_offset, s.seed = n_envs, int(env_offset), int(seed) & 0xFFFFFFFFFFFFFFFF
        s.episode, s.week = 0, -1
        s.inventory, s.backlog, s.orders_placed = self._inv.data_ptr(), self._bk.data_ptr(), self._op.data_ptr()
        s.shipments = self._ring.data_ptr()
        s.inventory_costs = self._inv_costs.data_ptr() if track_costs else None
        s.backlog_costs = self._bk_costs.data_ptr() if track_costs else None
        s.orders_history = self._hist.data_ptr() if track_history else None
        s.episode_return = self._ret.data_ptr() if track_returns else None
        s.final_return = self._final_ret.data_ptr() if track_returns else None
        s.penalty_costs = self._pen_costs.data_ptr() if self._pen_costs is not None else None
        s.error_flags = self._err.data_ptr()
        s.error_host = self._err_word.dev
        s.slab = self._slab.data_ptr() if self._slab is not None else None
        self._st = s
        self._cfg_ref = ctypes.byref(self._cfg)
        self._st_ref = ctypes.byref(self._st)
        self._done_flag = ctypes.c_int32(0)
        self._done_ref = ctypes.byref(self._done_flag)
        self._flags = nat.SCG_BG_AUTORESET if self.auto_reset else 0
        self._act_shape = (n_envs, L)
        self._obs_ptr, self._rew_ptr = self._obs.data_ptr(), self._rew.data_ptr()
        self._term_ptr = self._term_obs.data_ptr()
        self._cfg_addr, self._st_addr = ctypes.addressof(self._cfg), ctypes.addressof(self._st)
        self._fast_step, self._fast_step_timed = nat.fast.bg_step, nat.fast.bg_step_timed
        # the fixed arguments of a step behind one handle (scg_pybind.c bg_step_args): the
        # step loop passes three (flags are fixed per env; the rest are this env's buffers)
        self._step_args = nat.BgStepArgs(self._cfg_addr, self._st_addr, self._obs_ptr, self._rew_ptr, self._term_ptr,
                                         self._flags)
        self._step_handle = ctypes.addressof(self._step_args)
        self._fast_step_h = nat.fast.bg_step_h
        self._raw_stream = nat.raw_stream_fn()  # torch's current raw stream, one C call
        self._ready = {}  # id(actions) -> (weakref, data_ptr) of validated action tensors
        self._act_numel = n_envs * L
        # gym surface (an extension: the reference leaves both spaces unset, :62-64)
        self.single_observation_space = spaces.Box(_I32[0], _I32[1], (L,), np.int32)
        # actions: the reference's are unbounded int64 (:121); sampled ones stay within
        # +-ACTION_BOUND so an episode's int32 state cannot overflow (the error flag catches
        # any caller action that does)
        self.single_action_space = spaces.Box(-ACTION_BOUND, ACTION_BOUND - 1, (L,), np.int32)
        self.observation_space = spaces.Box(_I32[0], _I32[1], (n_envs, L), np.int32)
        self.action_space = spaces.Box(-ACTION_BOUND, ACTION_BOUND - 1, (n_envs, L), np.int32)

    # -------------------------------------------------------------------------------
    def _stream(self):
        return nat.raw_stream(self._dev_index)

    def reset(self):
        """Reset every env; the reset kernel also clears the int32-overflow word (and its
        host-mapped copy), so an overflow is scoped to the episodes since the last reset()."""
        nat.check(nat.lib.scg_bg_reset(self._cfg_ref, self._st_ref, self._obs.data_ptr(), self._stream()))
        return self._obs

    def seed(self, seed=None, seed_group=None):
        """New Philox key (fresh entropy for None; with `seed_group`, the group's rank 0
        entropy — a collective, see distributed.entropy_seed); the next reset() starts
        episode 0 again."""
        self._st.seed = _entropy_seed(seed, seed_group)
        self._st.episode, self._st.week = 0, -1

    def _actions(self, actions):
        N, L = self.n_envs, self.levels
        if not isinstance(actions, torch.Tensor):
            actions = torch.as_tensor(np.asarray(actions))
        if actions.dtype.is_floating_point:
            actions = actions.trunc()
        if actions.dtype != torch.int32 or actions.device != self.device:
            actions = actions.to(device=self.device, dtype=torch.int32)
        if actions.shape != (N, L):
            if actions.numel() != N * L:
                raise ValueError(f"actions must have shape ({N}, {L}), got {tuple(actions.shape)}")
            actions = actions.reshape(N, L)
        return actions.contiguous()

    def _is_ready(self, a):
        return (type(a) is torch.Tensor and a.dtype is torch.int32 and a.is_cuda
                and a.get_device() == self._dev_index and a.shape == self._act_shape and a.is_contiguous())

    def step(self, actions, _events=None):
        # a tensor validated once is recognised by identity and data pointer (the policy's
        # per-week action buffers are reused), skipping the per-call checks; still contiguous
        # with N * L elements catches the in-place metadata changes that keep the pointer
        # (t_(), as_strided_(), resize_() to fewer rows) — any contiguous int32 buffer of
        # N * L elements is read as [N, L], as _actions() reshapes it
        ok = self._ready.get(id(actions))
        if ok is not None and ok[0]() is actions and ok[1] == actions.data_ptr() and actions.is_contiguous() \
                and actions.numel() == self._act_numel:
            ptr = ok[1]
        else:
            if self._is_ready(actions):
                if len(self._ready) >= 64:
                    self._ready.clear()
                self._ready[id(actions)] = (weakref.ref(actions), actions.data_ptr())
            else:
                actions = self._actions(actions)
            ptr = actions.data_ptr()
        if _events is None:
            r = self._fast_step_h(self._step_handle, ptr, self._raw_stream(self._dev_index))
        else:  # (start, stop) hipEvent_t handles stamped with the kernel's own dispatch times
            r = self._fast_step_timed(self._cfg_addr, self._st_addr, ptr, self._obs_ptr,
                                      self._rew_ptr, self._term_ptr, self._flags, _events[0], _events[1],
                                      nat.raw_stream(self._dev_index))
        if r > 1:
            nat.check(r >> 1)
        if r & 1:
            self._poll_errors()
            info = {"terminal_observation": self._term_obs}
            if self._final_ret is not None:
                info["episode_return"] = self._final_ret
            return self._obs, self._rew, self._done_true, info
        return self._obs, self._rew, self._done_false, {}

    def _poll_errors(self):
        """At a terminal step: raise if the overflow word an earlier terminal launch exported
        to host-mapped memory is set (no synchronisation: a launch still in flight reports
        at a later terminal step, or check_errors() reports at once)."""
        if self._err_word.value:
            raise OverflowError("a BeerGame value left int32 range (the reference's int64 state would differ); "
                                "results since then are invalid")

    def check_errors(self):
        """Raise OverflowError if any step so far produced a value outside int32 (the
        reference computes in int64; beergame_env.py:33,35,130-132). Synchronises."""
        if int(self._err.item()):
            raise OverflowError("a BeerGame value left int32 range (the reference's int64 state would differ); "
                                "results since then are invalid")

    # checkpoint / resume (gym_supplychain_amd/checkpoint.py) ------------------
    def _ckpt_buffers(self):
        """Every device buffer a step reads or writes, by the reference's attribute names
        (beergame_env.py:44-60, 123, 131-132), plus the outputs of the last step."""
        return {"inventory": self._inv, "backlog": self._bk, "orders_placed": self._op, "shipments": self._ring,
                "inventory_costs": self._inv_costs, "backlog_costs": self._bk_costs,
                "penalty_costs": self._pen_costs, "orders_history": self._hist, "episode_return": self._ret,
                "final_return": self._final_ret, "terminal_observation": self._term_obs,
                "error_flags": self._err, "obs_reward": self._out}

    def _ckpt_fingerprint(self):
        T = self.max_weeks
        fp = ckpt.config_fingerprint(self._cfg)
        fp += [["n_envs", self.n_envs], ["env_offset", int(self._st.env_offset)], ["auto_reset", int(self.auto_reset)],
               ["shipment_delays", list(self._delays)], ["plan", list(self._plan)],
               ["customer_demand", list(self._demand) if self._demand is not None else None],
               ["poisson_lambda", repr(getattr(self, "poisson_lambda", None))], ["horizon", T]]
        return fp

    def state_dict(self):
        """Checkpoint of every env: the device state (cloned on the current stream, after
        every step already enqueued) and the Philox key, episode and week. torch.save it;
        load_state_dict() on an env built with the same arguments resumes bit for bit."""
        return ckpt.snapshot(type(self).__name__, self._ckpt_fingerprint(),
                             {"seed": self._st.seed, "episode": self._st.episode, "week": self._st.week},
                             self._ckpt_buffers())

    def load_state_dict(self, state):
        """Restore a state_dict() of an env of this class and configuration (ValueError
        otherwise); the copies are enqueued on the current stream."""
        bufs = self._ckpt_buffers()
        ckpt.check(state, type(self).__name__, self._ckpt_fingerprint(), bufs)
        cnt = ckpt.restore(state, bufs)
        self._st.seed, self._st.episode, self._st.week = cnt["seed"], cnt["episode"], cnt["week"]
        # the host-mapped copy of the overflow word follows the restored device word
        self._err_word.value = int(state["tensors"]["error_flags"].reshape(-1)[0])

    def rollout(self, actions, obs_out=None, rewards_out=None):
        """K weeks in as few launches as possible (state kept in registers).

        actions int32 [K, N, L] on device. Returns (obs [K, N, L], rewards [K, N]); with
        auto-reset the obs row of a terminal week is the reset observation, as in step().
        """
        if not isinstance(actions, torch.Tensor) or actions.device != self.device or actions.dtype != torch.int32:
            actions = torch.as_tensor(actions).to(device=self.device, dtype=torch.int32)
        actions = actions.contiguous()
        K = actions.shape[0]
        if tuple(actions.shape) != (K, self.n_envs, self.levels):
            raise ValueError(f"actions must be [K, {self.n_envs}, {self.levels}]")
        if obs_out is None:
            obs_out = torch.empty((K, self.n_envs, self.levels), dtype=torch.int32, device=self.device)
        if rewards_out is None:
            rewards_out = torch.empty((K, self.n_envs), dtype=torch.int32, device=self.device)
        nat.check(nat.lib.scg_bg_rollout(self._cfg_ref, self._st_ref, K, actions.data_ptr(), obs_out.data_ptr(),
                                         rewards_out.data_ptr(), self._flags, self._stream()))
        return obs_out, rewards_out

    def poisson_demand(self, episode=None):
        """The Poisson demand [T, N] the kernels draw for `episode` (default: current)."""
        if self.demand_mode != nat.SCG_DEMAND_POISSON:
            raise ValueError("env is not in poisson demand mode")
        out = torch.empty((self.max_weeks, self.n_envs), dtype=torch.int32, device=self.device)
        ep = self._st.episode if episode is None else int(episode)
        nat.check(nat.lib.scg_bg_poisson_demand(self._cfg_ref, self._st_ref, ep, out.data_ptr(), self._stream()))
        return out

    # state views (device tensors, reference attribute names) -------------------------
    @property
    def week(self):
        return self._st.week

    @property
    def episode(self):
        return self._st.episode

    @property
    def env_offset(self):
        return self._st.env_offset

    @property
    def seed_value(self):
        return self._st.seed

    @property
    def inventory(self):
        return self._inv

    @property
    def backlog(self):
        return self._bk

    @property
    def orders_placed(self):
        return self._op

    @property
    def inventory_costs(self):
        return self._inv_costs

    @property
    def backlog_costs(self):
        return self._bk_costs

    @property
    def penalty_costs(self):
        """BeerGameEnv2 only: [N, L] capacity-penalty ledger (beergame2_env.py:184)."""
        return self._pen_costs

    @property
    def all_orders_placed(self):
        """[N, L, T+1] like the reference's all_orders_placed (:123, :151-152)."""
        return None if self._hist is None else self._hist.permute(1, 2, 0)

    @property
    def episode_return(self):
        return self._ret

    @property
    def final_return(self):
        return self._final_ret

    @property
    def full_table(self):
        return bool(self._cfg.full_table)

    def scheduled_rows(self, week=None):
        """Bool [R]: the shipment-table rows the current episode has scheduled by `week`
        (default: now) — weeks 1..d0 of the initial pipeline (:52) and w + d_w for every
        week w <= `week` with d_w > 0 (:96, :114). Host arithmetic on the config only."""
        w = self.week if week is None else int(week)
        R, d = self.ring_slots, self.config.shipment_delays
        rows = np.zeros(R, dtype=bool)
        rows[1: 1 + int(d[0])] = True
        for k in range(1, max(w, 0) + 1):
            if d[k] > 0 and k + d[k] < R:
                rows[k + d[k]] = True
        return rows

    def shipment_table(self):
        """int64 [N, R, L]: the reference's absolute-week `shipments` table of every env
        (beergame_env.py:46-52, :96, :114) — needs full_table=True. Row s is week s; rows
        the episode has not scheduled yet read 0, as in the reference."""
        if not self._cfg.full_table:
            raise ValueError("shipment_table() needs BeerGameVecEnv(..., full_table=True)")
        t = self._ring.permute(1, 0, 2).to(torch.int64)
        mask = torch.as_tensor(self.scheduled_rows(), device=t.device)
        return t * mask.view(1, -1, 1)

    def close(self):
        pass


_SERVERS = {}  # (device index, levels, demand mode) -> _StepServer, one resident wave each


@atexit.register
def _stop_servers():  # no step-server wave outlives the interpreter (nor its mailbox)
    for sv in list(_SERVERS.values()):
        sv.close()


class _StepServer:
    """A step server (include/scgpu.h scg_bg_server_*): one wave on a non-blocking,
    high-priority stream of its own polls a mailbox in host-mapped memory and runs each week
    an attached env posts on that env's state. One per (device, levels, demand mode) in a
    process, whatever the number of drop-in envs (up to BG_SERVER_SLOTS per server; more
    start another server): many envs stepped in turn share one resident wave and one stream.
    The high priority puts the stream on a hardware queue of its own pool, so the parked wave
    never holds up work of normal-priority streams that would share its queue; and at most one
    server per device is resident at a time (envs/resident.py). The wave exits
    when stopped, or by itself after IDLE_US without a request; a post launches it again when
    needed. The mailbox is freed only after the wave has been stopped."""

    IDLE_US = 20000

    @classmethod
    def attach(cls, vec, act_dev, act_host, obs_dev, rew_dev):
        """A slot of this process's server for `vec` (a free one, or a new server)."""
        key0 = (vec._dev_index, int(vec._cfg.levels), int(vec._cfg.demand_mode))
        for j in range(64):
            key = key0 + (j,)
            sv = _SERVERS.get(key)
            if sv is None:
                sv = _SERVERS[key] = cls(vec.device, key0[1], key0[2], key)
            if bin(sv.sv.slots_used).count("1") < nat.BG_SERVER_SLOTS:
                return _ServerSlot(sv, vec, act_dev, act_host, obs_dev, rew_dev)
        raise RuntimeError("too many drop-in envs on one device for the step server")

    def __init__(self, device, levels, demand_mode, key):
        stream, self.priority = resident.server_stream(device)
        self._device, self._dev_index, self._key = device, key[0], key
        self._box = box = nat.MappedBuffer(ctypes.sizeof(nat.BgServerBox))
        self.box = nat.BgServerBox.from_address(box.host)
        self.sv = nat.BgServer(box.host, box.dev, stream, levels, demand_mode, self.IDLE_US, 0)
        self._closed = False

    @property
    def launches(self):
        return int(self.sv.launches)

    def stop(self):
        if not self._closed:
            with torch.cuda.device(self._device):
                nat.check(nat.lib.scg_bg_server_stop(ctypes.byref(self.sv)))

    def close(self):
        if self._closed:
            return
        self.stop()  # raises if the wave cannot be stopped: then the mailbox stays allocated
        self._closed = True
        resident.release(self._dev_index, self)
        resident.destroy_stream(self.sv.stream)
        self._box = None
        if _SERVERS.get(self._key) is self:
            del _SERVERS[self._key]


class _ServerSlot:
    """One drop-in env's slot of a _StepServer: step() posts the env's week and returns once
    the wave has written its observation and reward (scg_pybind.c bg_server_step)."""

    def __init__(self, server, vec, act_dev, act_host, obs_dev, rew_dev):
        self.server = server
        self.slot = nat.BgServerSlot(None, act_dev, act_host, obs_dev, rew_dev, -1)
        nat.check(nat.lib.scg_bg_server_attach(ctypes.byref(server.sv), ctypes.byref(self.slot)))
        self._args = (vec._cfg_addr, vec._st_addr, ctypes.addressof(self.slot))
        self._fast = nat.fast.bg_server_step
        self._claim = (server._dev_index, server)

    @property
    def sv(self):
        return self.server.sv

    def step(self):
        resident.claim(*self._claim)
        return self._fast(*self._args)

    def close(self):
        if self.slot.index >= 0 and not self.server._closed:
            nat.check(nat.lib.scg_bg_server_detach(ctypes.byref(self.slot)))

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter teardown
            pass


class BeerGameEnv(spaces.Env):
    """Drop-in for gym_supplychain.envs.BeerGameEnv (beergame_env.py:6-181), one env.

    Same constructor, reset()/step()/render()/close() and NumPy return types: reset()
    and step() give int64 observations, step() an np.int64 reward, a bool done and {}
    (:138). Stepping past the last week raises IndexError (:79 on customer_demand[T]).
    The week runs on the GPU as a batch of one; use BeerGameVecEnv for throughput.
    Each step is posted to a resident wave (the step server, include/scgpu.h
    scg_bg_server_*) rather than launched; every drop-in env of the process with the same
    levels on the same device shares that one wave (a slot each). The wave exits 20 ms after
    the last step of any of them, so a device-wide torch.cuda.synchronize() right after a
    step waits up to that long. SCG_BG_SERVER=0 launches the step kernel per step instead.
    State attributes (inventory, backlog, orders_placed, incoming_orders, shipments, the
    ledgers, all_orders_placed) are read back from the device when accessed.
    """

    def __init__(self, env_init_info={}, device=None):  # noqa: B006 - reference signature (:11)
        self.DEBUG = False
        cfg = BeerGameConfig(env_init_info)
        # the reference's whole absolute-week shipment table (:46-50), for any horizon and
        # delays; separate state buffers (not the slab), so the overflow word can live in
        # host-mapped memory below
        self._vec = BeerGameVecEnv(1, env_init_info, demand="fixed", device=device, auto_reset=False,
                                   track_costs=True, track_history=True, track_returns=False, config=cfg,
                                   full_table=True, state_slab=False)
        cfg = self._vec.config
        self.levels = L = cfg.levels
        self.inv_cost = cfg.inv_cost
        self.backlog_cost = cfg.backlog_cost
        self.customer_demand = cfg.customer_demand.astype(np.int64)
        self.initial_inventory = cfg.initial_inventory.astype(np.int64)
        self.max_weeks = cfg.max_weeks
        self.shipment_delays = cfg.shipment_delays.astype(np.int64)
        self.initial_shipment_value = cfg.initial_shipment_value
        self.initial_orders_value = cfg.initial_orders_value
        self.current_state = None
        # one host-mapped block for the step's inputs and outputs: the overflow word (the
        # kernel's plain store of 1, cleared by reset), the action row, and the observation
        # row + reward (profiles/r05*_facade_latency.log)
        ra = (4 * L + 15) // 16 * 16
        self._io = io = nat.MappedBuffer(16 + ra + 4 * (L + 1))
        self._err_np = io.view(np.int32, 0, 1)
        self._act_np = io.view(np.int32, 16, L)
        self._out_np = io.view(np.int32, 16 + ra, L + 1)
        self._act_dev = io.dev + 16
        vec = self._vec
        vec._st.error_flags = io.dev
        vec._err = torch.from_numpy(self._err_np)  # check_errors() reads the mapped word
        obs_dev, rew_dev = io.dev + 16 + ra, io.dev + 16 + ra + 4 * L
        # The week runs on a resident wave that polls the mailbox (scg_bg_server_step): no
        # launch and no stream synchronisation per step. SCG_BG_SERVER=0: one launch of the
        # step kernel plus one synchronisation per step instead.
        self._server = None
        if os.environ.get("SCG_BG_SERVER", "1") != "0":
            self._server = _StepServer.attach(self._vec, self._act_dev, io.host + 16, obs_dev, rew_dev)
        self._step_args = nat.BgStepArgs(vec._cfg_addr, vec._st_addr, obs_dev, rew_dev, vec._term_ptr, 0)
        self._handle = ctypes.addressof(self._step_args)
        self._fast_step_h = nat.fast.bg_step_h
        self._sync = nat.stream_synchronize_fn()
        self._last_act = None
        self.week = None

    def reset(self):
        # No request of this env is in flight (step() returns once it is answered), so the
        # shared wave may keep serving other envs while the reset kernel rewrites this one's
        # state; the next post publishes the new episode's arguments and the wave's acquire
        # per request reads the reset state.
        obs = self._vec.reset()
        self.week = 0
        self._last_act = None
        self.current_state = obs[0].cpu().numpy().astype(np.int64)  # waits for the reset kernel
        return self.current_state

    def step(self, action):
        if self.week is None:  # the reference has no `week` before reset() (:67)
            raise AttributeError("'BeerGameEnv' object has no attribute 'week' (call reset() first)")
        a = np.asarray(action)
        if a.dtype.kind == "f":
            a = np.trunc(a)
        if a.shape == self._act_np.shape:
            self._act_np[:] = a
        else:
            self._act_np[:] = np.broadcast_to(a, (self.levels,))
        if self._server is not None:
            r = self._server.step()  # returns once the wave has written obs and reward
            if r > 1:
                nat.check(r >> 1)
        else:
            stream = self._vec._raw_stream(self._vec._dev_index)
            r = self._fast_step_h(self._handle, self._act_dev, stream)
            if r > 1:
                nat.check(r >> 1)
            rc = self._sync(stream)
            if rc:
                raise RuntimeError(f"hipStreamSynchronize failed ({rc})")
        if int(self._err_np[0]):  # the reference's int64 values no longer fit the int32 state
            raise OverflowError("a BeerGame value left int32 range; the GPU state no longer matches the reference")
        L = self.levels
        self.week = self._vec.week
        self._last_act = self._act_np.astype(np.int64)
        self.current_state = self._out_np[:L].astype(np.int64)
        reward = np.int64(self._out_np[L])
        if self.DEBUG:
            print('env.step()', self.current_state)
        return self.current_state, reward, self.week == self.max_weeks, {}

    # reference attributes, read back from the device on access
    def _row(self, t):
        return t[0].cpu().numpy().astype(np.int64)

    @property
    def inventory(self):
        return self._row(self._vec.inventory)

    @property
    def backlog(self):
        return self._row(self._vec.backlog)

    @property
    def orders_placed(self):
        return self._row(self._vec.orders_placed)

    @property
    def inventory_costs(self):
        return self._row(self._vec.inventory_costs)

    @property
    def backlog_costs(self):
        return self._row(self._vec.backlog_costs)

    @property
    def all_orders_placed(self):
        return self._vec.all_orders_placed[0].cpu().numpy().astype(np.int64)

    @property
    def incoming_orders(self):
        """The order slips of the last week (:79-81): customer demand at level 0, the orders
        of the level below above it — the kernel's orders_placed minus the action it added
        (:121); the initial orders after reset() (:145)."""
        if self._last_act is None:
            return np.full(self.levels, self.initial_orders_value, dtype=np.int64)
        return self.orders_placed - self._last_act

    @property
    def shipments(self):
        """The reference's absolute-week table [rows, L] (:46-52): row w is what arrives in
        week w, past weeks included (the table is never shifted, :73-74)."""
        return self._vec.shipment_table()[0].cpu().numpy()

    def render(self, mode='human'):  # beergame_env.py:158-175
        inv, bk = self.inventory, self.backlog
        print('\n' + '=' * 20)
        print('Week:\t', self.week)
        print('Inventory:\t', inv, bk, inv - bk)
        print('Incoming order:\t', self.incoming_orders)
        print('Orders placed:\t', self.orders_placed)
        if self.week is not None and self.week < self.max_weeks:
            print('Next customer demand:\t', self.customer_demand[self.week])
        if self.week is not None:
            table = self.shipments
            print('Next shipments:\t', [(i, list(table[i])) for i in range(self.week + 1, self.week + 6)
                                        if i < len(table)])
        if self.week is not None:
            print('Current delay:\t', self.shipment_delays[self.week])
        print('Inventory costs:\t', self.inventory_costs)
        print('Backlog costs:\t', self.backlog_costs)

    def close(self):
        if self._server is not None:
            self._server.close()

    def __del__(self):
        server = getattr(self, "_server", None)
        if server is not None:
            server.close()

    def _observation(self):
        return self.inventory - self.backlog


# ----------------------------------------------------------------------------------------
# beergame-v2: BeerGameEnv2 (gym_supplychain/envs/beergame2_env.py:5-211)
def _is_range(x):
    """The reference reads a tuple, or a list of exactly two items, as a [low, high) range (:41, :51)."""
    return isinstance(x, tuple) or (isinstance(x, list) and len(x) == 2)


class _Bg2Config:
    """BeerGameEnv2.__init__ (:10-71) resolved for the kernels."""

    def __init__(self, max_stock, max_order, weeks, levels, customer_demand, initial_inventory, inv_cost, backlog_cost,
                 exceeded_capacity_penalty, shipment_delays, initial_shipment, initial_orders):
        self.levels = _int32("levels", levels)
        if not 1 <= self.levels <= nat.BG_MAX_LEVELS:
            raise ValueError(f"levels={self.levels} outside 1..{nat.BG_MAX_LEVELS}")
        self.max_weeks = _int32("weeks", weeks)
        if not 1 <= self.max_weeks <= nat.BG_MAX_WEEKS:
            raise ValueError(f"weeks={self.max_weeks} outside 1..{nat.BG_MAX_WEEKS}")
        self.max_stock = _int32("max_stock", max_stock)
        self.max_order = _int32("max_order", max_order)
        self.inv_cost, self.backlog_cost = _int32("inv_cost", inv_cost), _int32("backlog_cost", backlog_cost)
        self.penalty = _int32("exceeded_capacity_penalty", exceeded_capacity_penalty)
        self.initial_inventory = _int32_list("initial_inventory", initial_inventory)
        if self.initial_inventory.size != self.levels:
            raise ValueError(f"initial_inventory has {self.initial_inventory.size} entries, levels={self.levels}")
        self.initial_shipment_value = _int32("initial_shipment", initial_shipment)
        self.initial_orders_value = _int32("initial_orders", initial_orders)
        T = self.max_weeks
        self.demand_range = None
        if _is_range(customer_demand):
            self.demand_range = (_int32("demand low", customer_demand[0]), _int32("demand high", customer_demand[1]))
            if self.demand_range[1] <= self.demand_range[0]:
                raise ValueError("customer_demand range must have low < high")  # randint(low, high)
            self.customer_demand = np.zeros(T, dtype=np.int32)
        else:
            self.customer_demand = _int32_list("customer_demand", customer_demand)
            if self.customer_demand.size < T:
                raise IndexError(f"customer_demand has {self.customer_demand.size} weeks, weeks={T}")
        self.delay_range = None
        if isinstance(shipment_delays, (bool, np.bool_)):
            raise TypeError("shipment_delays must be an int, a (low, high) range or a list")
        if isinstance(shipment_delays, (int, np.integer)):
            self.shipment_delays = np.asarray([2] + [int(shipment_delays)] * T, dtype=np.int32)   # :50
        elif _is_range(shipment_delays):
            lo, hi = int(shipment_delays[0]), int(shipment_delays[1])
            if not 0 <= lo < hi <= nat.BG_MAX_DELAY + 1:
                raise ValueError(f"shipment delay range must satisfy 0 <= low < high <= {nat.BG_MAX_DELAY + 1}")
            self.delay_range = (lo, hi)
            self.shipment_delays = np.asarray([2] + [lo] * T, dtype=np.int32)
        else:
            self.shipment_delays = _int32_list("shipment_delays", [2] + list(shipment_delays))         # :55
            if self.shipment_delays.size < T + 1:
                raise IndexError(f"shipment_delays needs {T} entries")
            self.shipment_delays = self.shipment_delays[: T + 1].copy()
        if self.shipment_delays.min() < 0 or self.shipment_delays.max() > nat.BG_MAX_DELAY:
            raise ValueError(f"shipment delays must be within 0..{nat.BG_MAX_DELAY}")


class BeerGame2VecEnv(BeerGameVecEnv):
    """N lock-step BeerGameEnv2 envs: same keywords as the reference class (:10-14).

    Observations are int32 `max_stock + inventory - backlog`; actions are the absolute
    orders (int32 [N, L]); rewards include the capacity penalty. A (low, high)
    customer_demand or shipment_delays draws randint(low, high) per (env, episode, week)
    on device with Philox (streams 4 and 5) where the reference uses RandomState (:76-92).
    """

    def __init__(self, n_envs, max_stock=100, max_order=30, weeks=35, levels=4, customer_demand=None,
                 initial_inventory=(12, 12, 12, 12), inv_cost=1, backlog_cost=2, exceeded_capacity_penalty=100,
                 shipment_delays=2, initial_shipment=4, initial_orders=4, seed=None, device=None, env_offset=0,
                 auto_reset=True, track_costs=True, track_history=False, track_returns=True, seed_group=None):
        if customer_demand is None:
            customer_demand = [4] * 4 + [8] * 31
        cfg = _Bg2Config(max_stock, max_order, weeks, levels, customer_demand, list(initial_inventory), inv_cost,
                         backlog_cost, exceeded_capacity_penalty, shipment_delays, initial_shipment, initial_orders)
        fields = dict(variant=2, max_stock=cfg.max_stock, exceeded_capacity_penalty=cfg.penalty)
        if cfg.delay_range:
            fields.update(stochastic_delays=1, delay_lo=cfg.delay_range[0], delay_hi=cfg.delay_range[1])
        demand = ("uniform",) + cfg.demand_range if cfg.demand_range else "fixed"
        # seed=None: fresh entropy, as the reference's RandomState(None) (beergame2_env.py:58);
        # shards of one batch share rank 0's only when asked (seed_group, a collective)
        super().__init__(n_envs, None, demand=demand, seed=_entropy_seed(seed, seed_group), device=device,
                         env_offset=env_offset, auto_reset=auto_reset, track_costs=track_costs,
                         track_history=track_history, track_returns=track_returns, config=cfg, variant_fields=fields)
        self.max_stock, self.max_order = cfg.max_stock, cfg.max_order
        L = cfg.levels
        self.single_observation_space = spaces.Box(0, 2 * cfg.max_stock - 1, (L,), np.int32)   # MultiDiscrete (:28)
        self.single_action_space = spaces.Box(0, cfg.max_order - 1, (L,), np.int32)            # MultiDiscrete (:27)

    def rollout(self, *a, **k):
        raise NotImplementedError("rollout is not implemented for BeerGameEnv2")


class BeerGameEnv2(spaces.Env):
    """Drop-in for gym_supplychain.envs.BeerGameEnv2 (beergame2_env.py:5-211), one env.

    reset() -> int64 observation; step(action) -> (int64 obs, Python int reward, bool, {});
    inventory_costs / backlog_costs / penalty_costs are float64 like the reference's.
    """

    def __init__(self, max_stock=100, max_order=30, weeks=35, levels=4, customer_demand=[4] * 4 + [8] * 31,  # noqa: B006
                 initial_inventory=[12, 12, 12, 12], inv_cost=1, backlog_cost=2,  # noqa: B006
                 exceeded_capacity_penalty=100, shipment_delays=2, initial_shipment=4, initial_orders=4, seed=None,
                 device=None):
        self.DEBUG = False
        self._vec = BeerGame2VecEnv(1, max_stock, max_order, weeks, levels, customer_demand, initial_inventory,
                                    inv_cost, backlog_cost, exceeded_capacity_penalty, shipment_delays,
                                    initial_shipment, initial_orders, seed=seed, device=device, auto_reset=False,
                                    track_costs=True, track_history=True, track_returns=False)
        self.levels, self.max_stock, self.max_weeks = levels, max_stock, weeks
        self.action_space = spaces.MultiDiscrete(levels * [max_order])               # :27
        self.observation_space = spaces.MultiDiscrete(levels * [2 * max_stock])      # :28
        self.current_state = None
        self.week = None
        pin = torch.cuda.is_available()
        self._act_host = torch.zeros((1, levels), dtype=torch.int32, pin_memory=pin)
        self._act_np = self._act_host.numpy()
        self._act_dev = torch.zeros((1, levels), dtype=torch.int32, device=self._vec.device)
        self._out_host = torch.zeros(self._vec._out.shape, dtype=torch.int32, pin_memory=pin)
        self._out_np = self._out_host.numpy()

    def seed(self, seed=None):
        self._vec.seed(seed)

    def reset(self):
        obs = self._vec.reset()
        self.week = 0
        self.current_state = obs[0].cpu().numpy().astype(np.int64)
        return self.current_state

    def step(self, action):
        if self.week is None:
            raise AttributeError("'BeerGameEnv2' object has no attribute 'week' (call reset() first)")
        self._act_np[0, :] = np.asarray(action).astype(np.int64).reshape(-1)
        self._act_dev.copy_(self._act_host, non_blocking=True)
        self._vec.step(self._act_dev)
        self._out_host.copy_(self._vec._out, non_blocking=True)
        torch.cuda.current_stream(self._vec.device).synchronize()
        L = self.levels
        self.week = self._vec.week
        self.current_state = self._out_np[:L].astype(np.int64)
        return self.current_state, int(self._out_np[L]), self.week == self.max_weeks, {}

    def _row(self, t, dtype=np.int64):
        return t[0].cpu().numpy().astype(dtype)

    @property
    def inventory(self):
        return self._row(self._vec.inventory)

    @property
    def backlog(self):
        return self._row(self._vec.backlog)

    @property
    def orders_placed(self):
        return self._row(self._vec.orders_placed)

    @property
    def inventory_costs(self):
        return self._row(self._vec.inventory_costs, np.float64)

    @property
    def backlog_costs(self):
        return self._row(self._vec.backlog_costs, np.float64)

    @property
    def penalty_costs(self):
        return self._row(self._vec.penalty_costs, np.float64)

    @property
    def all_orders_placed(self):
        return self._vec.all_orders_placed[0].cpu().numpy().astype(np.int64)

    def render(self, mode='human'):
        inv, bk = self.inventory, self.backlog
        print('\n' + '=' * 20)
        print('Week:\t', self.week)
        print('Inventory/back:\t', inv, bk, inv - bk)
        print('Orders placed:\t', self.orders_placed)
        print('Inventory costs:', self.inventory_costs)
        print('Backlog costs:\t', self.backlog_costs)
        print('Penalty costs:\t', self.penalty_costs)

    def close(self):
        pass
