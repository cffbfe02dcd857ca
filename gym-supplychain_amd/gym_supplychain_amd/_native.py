"""ctypes binding of libscgpu.so, the C ABI declared in include/scgpu.h.

The library is built in-tree (``__graft_entry__.build()`` / ``python -m
gym_supplychain_amd.build``) next to this file. There is no CPU fallback: every env
in this package runs its dynamics through these entry points, and importing this
module raises when the library is missing or was built for another ABI.

torch is imported first on purpose: torch ships its own libamdhip64.so (soname
libamdhip64.so.7) and the dynamic loader then binds libscgpu.so to that same HIP
runtime, so torch's streams and allocations are valid handles for our kernels.
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime libscgpu.so binds to)

LIB_NAME = "libscgpu.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
ABI_VERSION = 7

SCG_OK = 0
SCG_ERR_INVALID = 1
SCG_ERR_PAST_HORIZON = 2
SCG_ERR_NOT_RESET = 3
SCG_ERR_HIP = 4
SCG_PENDING = 5  # scg_bg_server_wait: not answered yet (not an error)

SCG_DEMAND_FIXED = 0
SCG_DEMAND_TABLE = 1
SCG_DEMAND_POISSON = 2
SCG_DEMAND_UNIFORM = 3

SCG_BG_AUTORESET = 1
SCG_SC_SERIAL = 2  # node-parallel SupplyChain kernel: every env through its serial walk (tests)
SCG_STREAM_DEMAND = 0
SCG_STREAM_ACTION = 1
SCG_STREAM_BG2_DEMAND = 4
SCG_STREAM_BG2_DELAY = 5

BG_MAX_LEVELS = 16
BG_MAX_WEEKS = 4096
BG_MAX_DELAY = 4096
POISSON_MAX = 256
BG_ROLLOUT_MAX = 128

_i32p = ctypes.POINTER(ctypes.c_int32)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_i64p = ctypes.POINTER(ctypes.c_int64)


class BgConfig(ctypes.Structure):
    """scg_bg_config (include/scgpu.h)."""
    _fields_ = [
        ("levels", ctypes.c_int32),
        ("max_weeks", ctypes.c_int32),
        ("inv_cost", ctypes.c_int32),
        ("backlog_cost", ctypes.c_int32),
        ("initial_shipment_value", ctypes.c_int32),
        ("initial_orders_value", ctypes.c_int32),
        ("initial_inventory", ctypes.c_int32 * BG_MAX_LEVELS),
        ("demand_mode", ctypes.c_int32),
        ("poisson_len", ctypes.c_int32),
        ("shipment_delays", ctypes.c_void_p),
        ("customer_demand", ctypes.c_void_p),
        ("demand_table", ctypes.c_void_p),
        ("poisson_thresholds", ctypes.c_void_p),
        ("plan", ctypes.c_void_p),
        ("ring_slots", ctypes.c_int32),
        ("variant", ctypes.c_int32),
        ("max_stock", ctypes.c_int32),
        ("exceeded_capacity_penalty", ctypes.c_int32),
        ("demand_lo", ctypes.c_int32),
        ("demand_hi", ctypes.c_int32),
        ("stochastic_delays", ctypes.c_int32),
        ("delay_lo", ctypes.c_int32),
        ("delay_hi", ctypes.c_int32),
        ("full_table", ctypes.c_int32),
    ]


class BgState(ctypes.Structure):
    """scg_bg_state (include/scgpu.h)."""
    _fields_ = [
        ("n_envs", ctypes.c_int64),
        ("env_offset", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("episode", ctypes.c_uint32),
        ("week", ctypes.c_int32),
        ("inventory", ctypes.c_void_p),
        ("backlog", ctypes.c_void_p),
        ("orders_placed", ctypes.c_void_p),
        ("shipments", ctypes.c_void_p),
        ("inventory_costs", ctypes.c_void_p),
        ("backlog_costs", ctypes.c_void_p),
        ("orders_history", ctypes.c_void_p),
        ("episode_return", ctypes.c_void_p),
        ("final_return", ctypes.c_void_p),
        ("penalty_costs", ctypes.c_void_p),
        ("error_flags", ctypes.c_void_p),
        ("error_host", ctypes.c_void_p),
        ("slab", ctypes.c_void_p),
    ]


BG_SERVER_SLOTS = 15
BG_SERVER_ARGS_BYTES = 512


class BgServerLine(ctypes.Structure):
    """scg_bg_server_line (include/scgpu.h): one slot's 64-byte request line."""
    _fields_ = [("req_seq", ctypes.c_uint32), ("cmd", ctypes.c_int32), ("wpack", ctypes.c_uint32),
                ("week", ctypes.c_int32), ("demand_fixed", ctypes.c_int32), ("n_inline", ctypes.c_int32),
                ("gen", ctypes.c_uint32), ("check", ctypes.c_uint32), ("action", ctypes.c_int32 * 8)]


class BgServerBox(ctypes.Structure):
    """scg_bg_server_box (include/scgpu.h): the step server's mailbox, in host-mapped memory."""
    _fields_ = [("req", BgServerLine * (BG_SERVER_SLOTS + 1)), ("done_seq", ctypes.c_uint32 * 16),
                ("n_slots", ctypes.c_uint32), ("exit_req", ctypes.c_uint32), ("exit_seq", ctypes.c_uint32),
                ("pad", ctypes.c_uint32 * 13),
                ("args", (ctypes.c_ubyte * BG_SERVER_ARGS_BYTES) * BG_SERVER_SLOTS)]


class BgServer(ctypes.Structure):
    """scg_bg_server (include/scgpu.h): one resident wave serving up to BG_SERVER_SLOTS envs."""
    _fields_ = [("box_host", ctypes.c_void_p), ("box_dev", ctypes.c_void_p), ("stream", ctypes.c_void_p),
                ("levels", ctypes.c_int32), ("demand_mode", ctypes.c_int32), ("idle_us", ctypes.c_int32),
                ("check_us", ctypes.c_int32), ("lock", ctypes.c_int32), ("running", ctypes.c_int32),
                ("slots_used", ctypes.c_uint32), ("pad", ctypes.c_int32), ("last_ns", ctypes.c_int64),
                ("launches", ctypes.c_int64)]


class BgServerSlot(ctypes.Structure):
    """scg_bg_server_slot (include/scgpu.h): one env's slot of a step server."""
    _fields_ = [("server", ctypes.c_void_p), ("action", ctypes.c_void_p), ("action_host", ctypes.c_void_p),
                ("obs", ctypes.c_void_p), ("reward", ctypes.c_void_p), ("index", ctypes.c_int32),
                ("gen", ctypes.c_uint32), ("seq", ctypes.c_uint32), ("week", ctypes.c_int32),
                ("done", ctypes.c_int32), ("relaunches", ctypes.c_int32)]


class ScServerBox(ctypes.Structure):
    """scg_sc_server_box (include/scgpu.h): the SupplyChain step server's mailbox."""
    _fields_ = [("req_seq", ctypes.c_uint32), ("cmd", ctypes.c_int32), ("t", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("episode", ctypes.c_uint32), ("opts", ctypes.c_uint32), ("pad0", ctypes.c_int32),
                ("check", ctypes.c_uint32), ("pad1", ctypes.c_int32 * 8), ("action", ctypes.c_float * 16),
                ("done_seq", ctypes.c_uint32), ("exit_req", ctypes.c_uint32), ("exit_seq", ctypes.c_uint32),
                ("pad2", ctypes.c_uint32 * 13)]


class ScServer(ctypes.Structure):
    """scg_sc_server (include/scgpu.h): the SupplyChain step server of one drop-in env."""
    _fields_ = [("box_host", ctypes.c_void_p), ("box_dev", ctypes.c_void_p), ("stream", ctypes.c_void_p),
                ("action", ctypes.c_void_p), ("action_host", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("reward", ctypes.c_void_p), ("idle_us", ctypes.c_int32), ("check_us", ctypes.c_int32),
                ("reload", ctypes.c_int32), ("running", ctypes.c_int32), ("seq", ctypes.c_uint32), ("t", ctypes.c_int32),
                ("done", ctypes.c_int32), ("relaunches", ctypes.c_int32), ("last_ns", ctypes.c_int64),
                ("launches", ctypes.c_int64)]


# scg_bg_slab_field: word offsets of a BeerGame state slab (scg_bg_slab_layout)
(SLAB_ERROR, SLAB_INVENTORY, SLAB_BACKLOG, SLAB_ORDERS, SLAB_INV_COSTS, SLAB_BACKLOG_COSTS, SLAB_TERMINAL_OBS,
 SLAB_RING, SLAB_EPISODE_RETURN, SLAB_FINAL_RETURN, SLAB_HISTORY, SLAB_TOTAL, SLAB_FIELDS) = range(13)


SC_MAX_PRODUCTS = 16
SC_MAX_DESTS = 32
SC_MAX_INIT = 16
SC_MAX_NODES = 256
SC_MAX_LEVELS = 16
SC_LEDGER_KEYS = 8  # info["sc_episode"] categories (supplychain_env.py:416-417)
SC_LEDGER_NAMES = ("stock", "stock_pen", "supply", "process", "process_pen", "ship", "ship_pen", "unmet_dem")
SC_KERNEL_AUTO, SC_KERNEL_LANE, SC_KERNEL_LEVEL, SC_KERNEL_STAGED, SC_KERNEL_NODES = 0, 1, 2, 3, 4
SC_LAYOUT_ENV_FASTEST, SC_LAYOUT_ENV_MAJOR = 0, 1
SCG_STREAM_SC_DEMAND = 2
SCG_STREAM_SC_LEADTIME = 3

_PA = ctypes.c_int32 * SC_MAX_PRODUCTS


class ScNode(ctypes.Structure):
    """scg_sc_node (include/scgpu.h)."""
    _fields_ = [
        ("last_level", ctypes.c_int32), ("n_supply", ctypes.c_int32), ("n_ship", ctypes.c_int32),
        ("n_dests", ctypes.c_int32), ("processing_capacity", ctypes.c_int32), ("retailer_index", ctypes.c_int32),
        ("action_offset", ctypes.c_int32), ("leadtime_offset", ctypes.c_int32),
        ("supply_capacity", _PA), ("supply_cost", _PA), ("stock_capacity", _PA), ("stock_cost", _PA),
        ("processing_ratio", _PA), ("processing_cost", _PA), ("max_ship", _PA), ("initial_stock", _PA),
        ("n_init", _PA),
        ("init_time", (ctypes.c_int32 * SC_MAX_INIT) * SC_MAX_PRODUCTS),
        ("init_amount", (ctypes.c_int32 * SC_MAX_INIT) * SC_MAX_PRODUCTS),
        ("dests", ctypes.c_int32 * SC_MAX_DESTS), ("ship_capacity", ctypes.c_int32 * SC_MAX_DESTS),
        ("dest_costs", (ctypes.c_int32 * SC_MAX_DESTS) * SC_MAX_PRODUCTS),
        ("in_deg", ctypes.c_int32), ("in_base", ctypes.c_int32),
        ("in_slot", ctypes.c_int32 * SC_MAX_DESTS), ("in_stride", ctypes.c_int32 * SC_MAX_DESTS),
    ]


class ScConfig(ctypes.Structure):
    """scg_sc_config (include/scgpu.h)."""
    _fields_ = [(f, ctypes.c_int32) for f in (
        "n_nodes", "n_products", "n_retailers", "n_actions", "n_obs", "n_leadtimes", "total_time_steps",
        "avg_leadtime", "max_leadtime", "stochastic_leadtimes", "demand_lo", "demand_hi", "unmet_demand_cost",
        "exceeded_stock_capacity_cost", "exceeded_process_capacity_cost", "exceeded_ship_capacity_cost",
        "heap_capacity", "leadtime_poisson_len", "obs_f64", "max_dests")] + [
        ("nodes", ctypes.c_void_p), ("leadtime_poisson", ctypes.c_void_p), ("demand_table", ctypes.c_void_p),
        ("leadtime_table", ctypes.c_void_p)] + [
        (f, ctypes.c_int32) for f in ("kernel", "layout", "group", "n_levels")] + [
        ("level_start", ctypes.c_int32 * (SC_MAX_LEVELS + 1)), ("inbox_size", ctypes.c_int32),
        ("level_staged", ctypes.c_int32), ("demand_models", ctypes.c_int32)] + [
        (f, ctypes.c_int32 * SC_MAX_PRODUCTS) for f in ("demand_kind", "demand_lo_p", "demand_hi_p",
                                                        "demand_pert_lo", "demand_pert_n")] + [
        ("demand_off", ctypes.c_int64 * SC_MAX_PRODUCTS), ("demand_thr", ctypes.c_void_p),
        ("demand_base", ctypes.c_void_p)]


class ScState(ctypes.Structure):
    """scg_sc_state (include/scgpu.h)."""
    _fields_ = [("n_envs", ctypes.c_int64), ("env_offset", ctypes.c_int64), ("seed", ctypes.c_uint64),
                ("episode", ctypes.c_uint32), ("time_step", ctypes.c_int32)] + [
        (f, ctypes.c_void_p) for f in ("stock", "heap_tk", "heap_val", "heap_size", "episode_return",
                                       "final_return", "error_flags", "inbox_tk", "inbox_val", "ledger",
                                       "ledger_kind", "final_ledger", "final_ledger_kind", "ledger_part")]


# Every symbol include/scgpu.h declares, with its ctypes signature.
SIGNATURES = {
    "scg_abi_version": (ctypes.c_int, []),
    "scg_last_error": (ctypes.c_char_p, []),
    "scg_bg_struct_sizes": (ctypes.c_int, [ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]),
    "scg_poisson_table": (ctypes.c_int, [ctypes.c_double, _u32p, ctypes.c_int32]),
    "scg_bg_prepare": (ctypes.c_int, [ctypes.POINTER(BgConfig)]),
    "scg_bg_slab_layout": (ctypes.c_int, [ctypes.POINTER(BgConfig), ctypes.c_int64, ctypes.c_int32, _i64p]),
    "scg_bg_reset": (ctypes.c_int, [ctypes.POINTER(BgConfig), ctypes.POINTER(BgState), ctypes.c_void_p,
                                    ctypes.c_void_p]),
    "scg_bg_step": (ctypes.c_int, [ctypes.POINTER(BgConfig), ctypes.POINTER(BgState), ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                   _i32p, ctypes.c_void_p]),
    "scg_bg_step_timed": (ctypes.c_int, [ctypes.POINTER(BgConfig), ctypes.POINTER(BgState), ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                         _i32p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "scg_bg_server_attach": (ctypes.c_int, [ctypes.POINTER(BgServer), ctypes.POINTER(BgServerSlot)]),
    "scg_bg_server_detach": (ctypes.c_int, [ctypes.POINTER(BgServerSlot)]),
    "scg_bg_server_post": (ctypes.c_int, [ctypes.POINTER(BgConfig), ctypes.POINTER(BgState),
                                          ctypes.POINTER(BgServerSlot)]),
    "scg_bg_server_wait": (ctypes.c_int, [ctypes.POINTER(BgState), ctypes.POINTER(BgServerSlot), ctypes.c_int64,
                                          _i32p]),
    "scg_bg_server_step": (ctypes.c_int, [ctypes.POINTER(BgConfig), ctypes.POINTER(BgState),
                                          ctypes.POINTER(BgServerSlot), _i32p]),
    "scg_bg_server_stop": (ctypes.c_int, [ctypes.POINTER(BgServer)]),
    "scg_bg_server_line_check": (ctypes.c_uint32, [ctypes.POINTER(BgServerLine)]),
    "scg_bg_rollout": (ctypes.c_int, [ctypes.POINTER(BgConfig), ctypes.POINTER(BgState), ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.c_void_p]),
    "scg_bg_poisson_demand": (ctypes.c_int, [ctypes.POINTER(BgConfig), ctypes.POINTER(BgState),
                                             ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "scg_sc_struct_sizes": (ctypes.c_int, [ctypes.POINTER(ctypes.c_size_t)] * 3),
    "scg_sc_prepare": (ctypes.c_int, [ctypes.POINTER(ScConfig), ctypes.POINTER(ScNode)]),
    "scg_sc_reset": (ctypes.c_int, [ctypes.POINTER(ScConfig), ctypes.POINTER(ScState), ctypes.c_void_p,
                                    ctypes.c_void_p]),
    "scg_sc_step": (ctypes.c_int, [ctypes.POINTER(ScConfig), ctypes.POINTER(ScState), ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, _i32p,
                                   ctypes.c_void_p]),
    "scg_sc_draw_tables": (ctypes.c_int, [ctypes.POINTER(ScConfig), ctypes.POINTER(ScState), ctypes.c_uint32,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "scg_sc_nodes_max_blocks": (ctypes.c_int, [ctypes.c_int32]),
    "scg_sc_server_post": (ctypes.c_int, [ctypes.POINTER(ScConfig), ctypes.POINTER(ScState), ctypes.POINTER(ScServer)]),
    "scg_sc_server_wait": (ctypes.c_int, [ctypes.POINTER(ScConfig), ctypes.POINTER(ScState), ctypes.POINTER(ScServer),
                                          ctypes.c_int64, _i32p]),
    "scg_sc_server_step": (ctypes.c_int, [ctypes.POINTER(ScConfig), ctypes.POINTER(ScState), ctypes.POINTER(ScServer),
                                          _i32p]),
    "scg_sc_server_stop": (ctypes.c_int, [ctypes.POINTER(ScServer)]),
    "scg_stream_copy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.c_void_p]),
    "scg_uniform_ints": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                        ctypes.c_int32, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p]),
}


class NativeLibraryError(ImportError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(gym_supplychain_amd has no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.scg_abi_version() != ABI_VERSION:
        raise NativeLibraryError(f"{LIB_PATH} ABI {lib.scg_abi_version()} != expected {ABI_VERSION}; rebuild it")
    cs, ss = ctypes.c_size_t(), ctypes.c_size_t()
    lib.scg_bg_struct_sizes(ctypes.byref(cs), ctypes.byref(ss))
    if (cs.value, ss.value) != (ctypes.sizeof(BgConfig), ctypes.sizeof(BgState)):
        raise NativeLibraryError(f"struct layout mismatch: C ({cs.value}, {ss.value}) vs ctypes "
                                 f"({ctypes.sizeof(BgConfig)}, {ctypes.sizeof(BgState)})")
    ns, cs, ss = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    lib.scg_sc_struct_sizes(ctypes.byref(ns), ctypes.byref(cs), ctypes.byref(ss))
    want = (ctypes.sizeof(ScNode), ctypes.sizeof(ScConfig), ctypes.sizeof(ScState))
    if (ns.value, cs.value, ss.value) != want:
        raise NativeLibraryError(f"SupplyChain struct layout mismatch: C {(ns.value, cs.value, ss.value)} vs {want}")
    return lib


lib = _load()

try:  # METH_FASTCALL binding of the per-step entry points (links this same libscgpu.so)
    from . import _scgpu_fast as fast
except ImportError as exc:  # pragma: no cover - built together with libscgpu.so
    raise NativeLibraryError(f"_scgpu_fast binding missing next to {LIB_PATH}: rebuild ({exc})")


def last_error():
    msg = lib.scg_last_error()
    return msg.decode() if msg else ""


def check(rc):
    """Map an scg_status to the exception the reference raises for the same misuse."""
    if rc == SCG_OK:
        return
    msg = last_error()
    if rc == SCG_ERR_INVALID:
        raise ValueError(msg)
    if rc == SCG_ERR_PAST_HORIZON:
        raise IndexError(msg)
    raise RuntimeError(msg or f"scgpu error {rc}")


def poisson_table(lam):
    """uint32 CDF thresholds for Poisson(lam), as a Python list (scg_poisson_table)."""
    buf = (ctypes.c_uint32 * POISSON_MAX)()
    n = lib.scg_poisson_table(float(lam), buf, POISSON_MAX)
    if n < 0:
        check(-n)
    return list(buf[:n])


try:  # the raw hipStream_t of torch's current stream without building a Stream object
    _raw_stream = torch._C._cuda_getCurrentRawStream
except AttributeError:  # pragma: no cover - older torch
    _raw_stream = None


class BgStepArgs(ctypes.Structure):
    """The fixed arguments of a BeerGame step (scg_pybind.c bg_step_args): addresses of the
    config and state structs and of the output buffers, and the step flags."""
    _fields_ = [("cfg", ctypes.c_uint64), ("state", ctypes.c_uint64), ("obs", ctypes.c_uint64),
                ("reward", ctypes.c_uint64), ("terminal_obs", ctypes.c_uint64), ("flags", ctypes.c_uint32)]


def raw_stream(device_index):
    if _raw_stream is not None:
        return _raw_stream(device_index)
    return torch.cuda.current_stream(device_index).cuda_stream


def raw_stream_fn():
    """raw_stream itself, or torch's C entry point when present (no Python frame per call)."""
    return _raw_stream if _raw_stream is not None else raw_stream


_hip = None


def hip_runtime():
    """The HIP runtime library torch loaded (so events/streams are shared handles)."""
    global _hip
    if _hip is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        _hip = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so.7")
        _hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        _hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        _hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
    return _hip


class MappedBuffer:
    """Pinned host memory the GPU reads and writes directly (hipHostMalloc, mapped and
    coherent): `host` / `dev` are its host and device addresses, `view(dtype, offset,
    count)` a NumPy array over part of it. The single-env facades put their action,
    observation and reward there, so a step is one launch and one stream synchronisation
    with no copies (the kernel's loads and stores cross PCIe)."""

    def __init__(self, nbytes):
        hip = hip_runtime()
        hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        hip.hipHostFree.argtypes = [ctypes.c_void_p]
        hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
        self.nbytes = max(64, (int(nbytes) + 63) // 64 * 64)
        host = ctypes.c_void_p()
        # hipHostMallocMapped | hipHostMallocCoherent: the kernel's stores reach the host
        # without depending on HIP_HOST_COHERENT
        if hip.hipHostMalloc(ctypes.byref(host), self.nbytes, 0x2 | 0x40000000) != 0:
            raise RuntimeError("hipHostMalloc failed")
        dev = ctypes.c_void_p()
        if hip.hipHostGetDevicePointer(ctypes.byref(dev), host, 0) != 0:
            hip.hipHostFree(host)
            raise RuntimeError("hipHostGetDevicePointer failed")
        self._hip, self.host, self.dev = hip, host.value, dev.value
        ctypes.memset(self.host, 0, self.nbytes)

    def view(self, dtype, offset, count):
        import numpy as np
        dt = np.dtype(dtype)
        if offset < 0 or offset % dt.itemsize or offset + count * dt.itemsize > self.nbytes:
            raise ValueError("view outside the mapped buffer")
        buf = (ctypes.c_char * (count * dt.itemsize)).from_address(self.host + offset)
        return np.frombuffer(buf, dtype=dt, count=count)

    def __del__(self):
        try:
            self._hip.hipHostFree(ctypes.c_void_p(self.host))
        except Exception:  # pragma: no cover - interpreter teardown
            pass


def stream_synchronize_fn():
    """hipStreamSynchronize(raw stream) -> int, one ctypes call."""
    hip = hip_runtime()
    f = hip.hipStreamSynchronize
    f.argtypes = [ctypes.c_void_p]
    f.restype = ctypes.c_int
    return f


class MappedWord:
    """One int32 of pinned host memory the GPU can write (hipHostMalloc, mapped): `dev` is
    its device address for kernels, `value` reads it on the host without synchronising."""

    def __init__(self):
        hip = hip_runtime()
        hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        hip.hipHostFree.argtypes = [ctypes.c_void_p]
        hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
        host = ctypes.c_void_p()
        # hipHostMallocMapped | hipHostMallocCoherent: the kernel's store reaches the host
        # without depending on HIP_HOST_COHERENT
        if hip.hipHostMalloc(ctypes.byref(host), 64, 0x2 | 0x40000000) != 0:
            raise RuntimeError("hipHostMalloc failed")
        dev = ctypes.c_void_p()
        if hip.hipHostGetDevicePointer(ctypes.byref(dev), host, 0) != 0:
            hip.hipHostFree(host)
            raise RuntimeError("hipHostGetDevicePointer failed")
        self._hip, self.host, self.dev = hip, host.value, dev.value
        self._word = ctypes.c_int32.from_address(self.host)
        self._word.value = 0

    @property
    def value(self):
        return self._word.value

    @value.setter
    def value(self, v):
        self._word.value = int(v)

    def __del__(self):
        try:
            self._hip.hipHostFree(ctypes.c_void_p(self.host))
        except Exception:  # pragma: no cover - interpreter teardown
            pass


def hip_event():
    """A new timing-enabled hipEvent_t (int handle) from torch's HIP runtime."""
    h = ctypes.c_void_p()
    if hip_runtime().hipEventCreate(ctypes.byref(h)) != 0:
        raise RuntimeError("hipEventCreate failed")
    return h.value


def hip_event_elapsed_ms(start, stop):
    ms = ctypes.c_float()
    rc = hip_runtime().hipEventElapsedTime(ctypes.byref(ms), start, stop)
    if rc != 0:
        raise RuntimeError(f"hipEventElapsedTime failed ({rc})")
    return ms.value


def hip_event_destroy(ev):
    hip_runtime().hipEventDestroy(ev)


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)
