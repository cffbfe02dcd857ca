"""The SupplyChain kernel body (scg_supplychain_core.h), compiled for the HOST by the
test-only harness tests/native/sc_host_harness.cpp, against the reference's golden
vectors: observations, rewards, stocks and heap storage order, bit for bit. This checks
the exact arithmetic the GPU kernel runs (NumPy-2 promotion emulation, heapq
restatement, Philox draws) on the CPU suite; the GPU parity tests repeat it on device.
"""
import numpy as np
import pytest

from golden_io import load_sc, sc_cases

CASES = sc_cases()


@pytest.fixture(scope="module")
def harness():
    import native_harness
    return native_harness.build()


def _setup(g, kernel=0):
    import ctypes
    from gym_supplychain_amd import _native as nat
    from gym_supplychain_amd.envs import SupplyChainSpec
    meta = g["meta"]
    spec = SupplyChainSpec(meta["nodes_info"], **meta["kwargs"])
    nodes = spec.node_table()
    c = nat.ScConfig()
    c.n_nodes, c.n_products, c.n_retailers = len(spec.nodes), spec.P, spec.n_retailers
    c.total_time_steps, c.avg_leadtime, c.max_leadtime = spec.total_time_steps, spec.avg_leadtime, spec.max_leadtime
    c.stochastic_leadtimes = int(spec.stochastic_leadtimes)
    from gym_supplychain_amd.envs import demand
    models = spec.demand_models
    c.demand_lo, c.demand_hi = models[0].lo, models[0].hi
    keep = []

    def host_upload(a):  # the host build reads the model tables from host memory
        keep.append(a)
        return a.ctypes.data

    if any(m.kind != demand.UNIFORM or (m.lo, m.hi) != (models[0].lo, models[0].hi) for m in models):
        demand.fill_config(c, models, spec.total_time_steps, host_upload)
    c._keep = keep
    for k, v in spec.penalties.items():
        setattr(c, k, v)
    thr = None
    if spec.stochastic_leadtimes:
        thr = nat.poisson_table(spec.avg_leadtime - 1)
        c.leadtime_poisson_len = len(thr)
    c.kernel = kernel
    assert nat.lib.scg_sc_prepare(ctypes.byref(c), nodes) == 0, nat.last_error()
    return spec, c, nodes, thr


@pytest.mark.parametrize("kernel", ["lane", "level"])
@pytest.mark.parametrize("name", CASES)
def test_host_build_of_kernel_body_matches_reference(harness, name, kernel):
    """Both kernels' step bodies: the lane kernel's serial chain walk and the level
    kernel's phases (scg_supplychain_level.h) with the group's lanes run in turn."""
    import native_harness
    from gym_supplychain_amd import _native as nat
    g = load_sc(name)
    meta = g["meta"]
    spec, c, nodes, thr = _setup(g, nat.SC_KERNEL_LANE if kernel == "lane" else nat.SC_KERNEL_LEVEL)
    N = g["obs"].shape[1]
    P, H = spec.P, c.heap_capacity
    for n in range(N):
        rc, obs, rew, stock, (tk, val, size) = native_harness.run_episode(harness, c, nodes, thr, meta["seed"], n, 0,
                                                                           g["actions"][:, n], kernel == "level")
        assert rc == 0
        assert np.array_equal(obs, g["obs"][:, n]), name
        assert np.array_equal(rew, g["reward"][:, n]), name
        assert np.array_equal(stock.reshape(stock.shape[0], -1, P), g["stock"][:, n])
        gt = g["heap_t"][:, n].reshape(len(obs), -1, g["heap_t"].shape[-1])
        gv = g["heap_v"][:, n].reshape(gt.shape)
        for s in range(len(obs)):
            for hp in range(gt.shape[1]):
                k = int(size[s, hp])
                assert k == int((gt[s, hp] >= 0).sum())
                assert (tk[s, hp, :k] >> 3).tolist() == gt[s, hp, :k].tolist()
                assert val[s, hp, :k].tolist() == gv[s, hp, :k].tolist()
        assert H >= gt.shape[-1]


@pytest.mark.parametrize("name", CASES)
def test_host_build_ledgers_match_reference(harness, name):
    """build_info: the kernel body's ledger notes (sc_note) against info['sc_episode'] as the
    reference recorded it after every step — values and NumPy types, exactly."""
    import native_harness
    from gym_supplychain_amd import _native as nat
    g = load_sc(name)
    meta = g["meta"]
    spec, c, nodes, thr = _setup(g, nat.SC_KERNEL_LANE)
    for n in range(g["obs"].shape[1]):
        rc, obs, rew, _, _, (led_v, led_k) = native_harness.run_episode(harness, c, nodes, thr, meta["seed"], n, 0,
                                                                       g["actions"][:, n], ledger=True)
        assert rc == 0
        assert np.array_equal(led_v[:, 0], g["led_cost"][:, n]) and np.array_equal(led_v[:, 1], g["led_units"][:, n])
        assert np.array_equal(led_k[:, 0], g["led_cost_k"][:, n]), name
        assert np.array_equal(led_k[:, 1], g["led_units_k"][:, n]), name
        assert np.allclose(np.cumsum(rew), g["led_rewards"][:, n], rtol=1e-12, atol=0)


@pytest.fixture(scope="module")
def harness_shipbits():
    import native_harness
    return native_harness.build(("SCG_STAGED_SHIP_BITS=1",))


@pytest.mark.parametrize("shipbits", [False, True])
@pytest.mark.parametrize("name", CASES)
def test_host_build_of_staged_kernel_matches_reference(harness, harness_shipbits, name, shipbits):
    """sc_step_staged_kernel's body (scg_supplychain_staged.h): one node's heaps staged at a
    time, shipments through the inbox — observations, rewards, stocks, heap storage order
    and ledgers against the reference, exactly; also with the ship capacities kept as
    overflow bits (SCG_STAGED_SHIP_BITS=1)."""
    import native_harness
    from gym_supplychain_amd import _native as nat
    g = load_sc(name)
    meta = g["meta"]
    spec, c, nodes, thr = _setup(g, nat.SC_KERNEL_STAGED)
    assert c.kernel == nat.SC_KERNEL_STAGED and c.inbox_size > 0
    P = spec.P
    for n in range(g["obs"].shape[1]):
        rc, obs, rew, stock, (tk, val, size), (led_v, led_k) = native_harness.run_episode(
            harness_shipbits if shipbits else harness, c, nodes, thr, meta["seed"], n, 0, g["actions"][:, n],
            staged=True)
        assert rc == 0
        assert np.array_equal(obs, g["obs"][:, n]), name
        assert np.array_equal(rew, g["reward"][:, n]), name
        assert np.array_equal(stock.reshape(stock.shape[0], -1, P), g["stock"][:, n])
        gt = g["heap_t"][:, n].reshape(len(obs), -1, g["heap_t"].shape[-1])
        gv = g["heap_v"][:, n].reshape(gt.shape)
        for s_ in range(len(obs)):
            for hp in range(gt.shape[1]):
                k = int(size[s_, hp])
                assert (tk[s_, hp, :k] >> 3).tolist() == gt[s_, hp, :k].tolist()
                assert val[s_, hp, :k].tolist() == gv[s_, hp, :k].tolist()
        assert np.array_equal(led_v[:, 0], g["led_cost"][:, n]) and np.array_equal(led_k[:, 1], g["led_units_k"][:, n])


@pytest.mark.parametrize("serial", [False, True])
@pytest.mark.parametrize("name", CASES)
def test_host_build_of_node_parallel_kernel_matches_reference(harness, name, serial):
    """sc_step_nodes_kernel's phases (scg_supplychain_nodes.h) with the nodes run in REVERSE
    order — every heap staged and its release summed without popping, every node acting on
    that, every heap then replaying its pushes and pops — against the reference, exactly.
    The inbox layout is the staged kernel's (the same scg_sc_prepare pass), so chains too
    wide for the kernel's LDS are checked too. serial=True runs every step through the
    kernel's fallback for unprovable receive orders (sc_nodes_serial) instead."""
    import native_harness
    from gym_supplychain_amd import _native as nat
    g = load_sc(name)
    meta = g["meta"]
    spec, c, nodes, thr = _setup(g, nat.SC_KERNEL_STAGED)
    P = spec.P
    harness.sch_nodes_fallbacks()
    for n in range(g["obs"].shape[1]):
        rc, obs, rew, stock, (tk, val, size) = native_harness.run_episode(
            harness, c, nodes, thr, meta["seed"], n, 0, g["actions"][:, n], nodes_kernel=True, nodes_serial=serial)
        assert rc == 0
        assert np.array_equal(obs, g["obs"][:, n]), name
        assert np.array_equal(rew, g["reward"][:, n]), name
        assert np.array_equal(stock.reshape(stock.shape[0], -1, P), g["stock"][:, n])
        gt = g["heap_t"][:, n].reshape(len(obs), -1, g["heap_t"].shape[-1])
        gv = g["heap_v"][:, n].reshape(gt.shape)
        for s_ in range(len(obs)):
            for hp in range(gt.shape[1]):
                k = int(size[s_, hp])
                assert (tk[s_, hp, :k] >> 3).tolist() == gt[s_, hp, :k].tolist()
                assert val[s_, hp, :k].tolist() == gv[s_, hp, :k].tolist()
    # the one-lane fallback is for amounts NumPy ties at float32 precision: none in these cases
    assert harness.sch_nodes_fallbacks() == 0, name


@pytest.mark.parametrize("serial", [False, True])
@pytest.mark.parametrize("name", CASES)
def test_host_build_of_node_parallel_ledgers_match_reference(harness, name, serial):
    """build_info in the node-parallel kernel: each node's act stores its entries in slots of
    its own (the nodes act at once, in reverse order here), and the step's ledger adds them
    in node order afterwards (sc_ledger_reduce, :750-760) — values and NumPy types of every
    entry against the reference after every step, exactly."""
    import native_harness
    from gym_supplychain_amd import _native as nat
    g = load_sc(name)
    meta = g["meta"]
    spec, c, nodes, thr = _setup(g, nat.SC_KERNEL_STAGED)
    for n in range(g["obs"].shape[1]):
        rc, obs, rew, _, _, (led_v, led_k) = native_harness.run_episode(
            harness, c, nodes, thr, meta["seed"], n, 0, g["actions"][:, n], ledger=True, nodes_kernel=True,
            nodes_serial=serial)
        assert rc == 0
        assert np.array_equal(obs, g["obs"][:, n]), name
        assert np.array_equal(led_v[:, 0], g["led_cost"][:, n]) and np.array_equal(led_v[:, 1], g["led_units"][:, n])
        assert np.array_equal(led_k[:, 0], g["led_cost_k"][:, n]), name
        assert np.array_equal(led_k[:, 1], g["led_units_k"][:, n]), name


def test_recv_scan_flags_float32_ties():
    """sc_recv_scan's fallback condition: two due amounts NumPy compares as equal (a float32
    against a Python float, compared in float32) with different doubles make the heappop
    order depend on the heap's shape, so the node-parallel kernel must not sum them itself."""
    import ctypes
    import native_harness
    lib = native_harness.build()
    f = lib.sch_recv_scan
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]

    def scan(entries, t):
        tk = np.array([(tt << 3) | k for tt, k, _ in entries], dtype=np.int32)
        v = np.array([x for _, _, x in entries], dtype=np.float64)
        out = ctypes.c_double()
        ok = f(tk.ctypes.data, v.ctypes.data, len(entries), t, ctypes.byref(out))
        return ok, out.value
    F32, PYF, F64, INT = 3, 1, 7, 0
    third32 = float(np.float32(1 / 3))
    assert scan([(5, F32, 0.5), (5, F64, 0.25), (6, F32, 9.0)], 5) == (1, 0.25 + 0.5)
    assert scan([(5, F32, third32), (5, PYF, 1 / 3)], 5)[0] == 0       # tied in float32, doubles differ
    assert scan([(5, F64, third32), (5, PYF, 1 / 3)], 5)[0] == 1       # compared exactly: ordered
    assert scan([(5, F32, 2.0), (5, INT, 2.0)], 5) == (1, 4.0)          # tied, same double
    assert scan([(4, F32, 1.0), (5, F32, 2.0)], 5)[0] == 0              # overdue entry


def test_auto_kernel_choice():
    """kernel='auto' (scg_sc_prepare, host only): the node-parallel kernel when every node
    gets a wave and two blocks fit a CU's LDS (2-per-stage), or one block does where the lane
    kernel's heaps would not fit LDS (the two-product 2-per-stage chain), the lane kernel
    with heaps in LDS when only a block's heaps fit (2-per-stage with max lead time 4: heaps
    of 10), the node-staged kernel on the wide ntom chain and the 3-product chain."""
    from gym_supplychain_amd import _native as nat
    _, c, _, _ = _setup(load_sc("2perstage"), nat.SC_KERNEL_AUTO)
    assert c.kernel == nat.SC_KERNEL_NODES and c.inbox_size > 0 and c.group == 8
    _, c, _, _ = _setup(load_sc("multiproduct"), nat.SC_KERNEL_AUTO)
    assert c.kernel == nat.SC_KERNEL_NODES and c.n_products == 2 and c.group == 8
    _, c, _, _ = _setup(load_sc("byproduct"), nat.SC_KERNEL_AUTO)
    assert c.kernel == nat.SC_KERNEL_STAGED and c.n_products == 3
    _, c, _, _ = _setup(load_sc("2perstage_stoch"), nat.SC_KERNEL_AUTO)
    assert c.kernel == nat.SC_KERNEL_LANE and c.inbox_size == 0
    _, c, _, _ = _setup(load_sc("ntom"), nat.SC_KERNEL_AUTO)
    assert c.kernel == nat.SC_KERNEL_STAGED and c.inbox_size > 0


@pytest.mark.parametrize("lt", [30, 31])
def test_staged_kernel_takes_lead_times_its_bytes_hold(lt):
    """The staged kernel's byte-packed entries hold times up to 30 steps after the step's own
    (scg_supplychain_staged.h): scg_sc_prepare refuses kernel='staged' past that, and
    kernel='auto' never picks it there."""
    import ctypes
    from gym_supplychain_amd import _native as nat
    from gym_supplychain_amd.envs import SupplyChainSpec
    meta = load_sc("2perstage")["meta"]
    kw = dict(meta["kwargs"], stochastic_leadtimes=False, avg_leadtime=lt, max_leadtime=lt)
    spec = SupplyChainSpec(meta["nodes_info"], **kw)
    for kernel in (nat.SC_KERNEL_STAGED, nat.SC_KERNEL_AUTO):
        c = nat.ScConfig()
        c.n_nodes, c.n_products, c.n_retailers = len(spec.nodes), spec.P, spec.n_retailers
        c.total_time_steps, c.avg_leadtime, c.max_leadtime = spec.total_time_steps, lt, lt
        c.demand_lo, c.demand_hi = spec.demand_models[0].lo, spec.demand_models[0].hi
        for k, v in spec.penalties.items():
            setattr(c, k, v)
        c.kernel = kernel
        rc = nat.lib.scg_sc_prepare(ctypes.byref(c), spec.node_table())
        if kernel == nat.SC_KERNEL_STAGED:
            if lt <= 30:
                assert rc == 0 and c.kernel == nat.SC_KERNEL_STAGED, nat.last_error()
            else:
                assert rc == nat.SCG_ERR_INVALID and "lead times" in nat.last_error()
        else:
            assert rc == 0 and (lt <= 30 or c.kernel != nat.SC_KERNEL_STAGED)


@pytest.mark.parametrize("init_time", [30, 31, 0, 64])
def test_initial_pipeline_times_bound_the_staged_kernel(init_time):
    """A C-ABI caller's initial pipeline times (the reference's reset uses 1..k, :402-412):
    the staged kernel's byte-packed entries hold times up to 30 after the step's, so a time
    past that makes scg_sc_prepare refuse kernel='staged' and kernel='auto' pick another
    kernel; a time outside 1..SCG_SC_MAX_INIT + lead time is refused by every kernel."""
    import ctypes
    from gym_supplychain_amd import _native as nat
    from gym_supplychain_amd.envs import SupplyChainSpec
    meta = load_sc("2perstage")["meta"]
    kw = dict(meta["kwargs"], stochastic_leadtimes=False, avg_leadtime=20, max_leadtime=20)
    spec = SupplyChainSpec(meta["nodes_info"], **kw)
    for kernel in (nat.SC_KERNEL_STAGED, nat.SC_KERNEL_AUTO, nat.SC_KERNEL_LANE):
        nodes = spec.node_table()
        nodes[3].init_time[0][0] = init_time
        c = nat.ScConfig()
        c.n_nodes, c.n_products, c.n_retailers = len(spec.nodes), spec.P, spec.n_retailers
        c.total_time_steps, c.avg_leadtime, c.max_leadtime = spec.total_time_steps, 20, 20
        c.demand_lo, c.demand_hi = spec.demand_models[0].lo, spec.demand_models[0].hi
        for k, v in spec.penalties.items():
            setattr(c, k, v)
        c.kernel = kernel
        rc = nat.lib.scg_sc_prepare(ctypes.byref(c), nodes)
        if not 1 <= init_time <= 16 + 20:
            assert rc == nat.SCG_ERR_INVALID and "initial pipeline time" in nat.last_error()
        elif kernel == nat.SC_KERNEL_STAGED and init_time > 30:
            assert rc == nat.SCG_ERR_INVALID and "lead times" in nat.last_error()
        else:
            assert rc == 0, nat.last_error()
            assert init_time <= 30 or c.kernel != nat.SC_KERNEL_STAGED
