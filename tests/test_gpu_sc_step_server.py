"""GPU tests of the drop-in SupplyChainEnv's step server (include/scgpu.h scg_sc_server_*: one
resident block of the node-parallel kernel's shape polling a host-mapped mailbox). Every
result is compared, bit for bit, with the launch path (SCG_SC_SERVER=0: one launch of the same
kernel and one synchronisation per step), which test_gpu_supplychain.py and
test_reference_pins.py pin to the reference."""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(monkeypatch, T=40, seed=11, **extra):
    from gym_supplychain_amd import SupplyChainEnv
    from gym_supplychain_amd.envs.scenarios import two_per_stage_nodes
    nodes, kw = two_per_stage_nodes(total_time_steps=T, **extra)
    kw.pop("seed", None)
    monkeypatch.setenv("SCG_SC_SERVER", "1")
    srv = SupplyChainEnv(nodes, seed=seed, **kw)
    monkeypatch.setenv("SCG_SC_SERVER", "0")
    ref = SupplyChainEnv(nodes, seed=seed, **kw)
    assert srv._server is not None and ref._server is None and srv._vec.kernel == ref._vec.kernel == "nodes"
    return srv, ref


def _same(srv, ref, act, where):
    o1, r1, d1, i1 = srv.step(act)
    o2, r2, d2, i2 = ref.step(act)
    assert np.array_equal(o1, o2) and r1 == r2 and d1 == d2 and i1 == i2, where
    assert srv.time_step == ref.time_step, where
    return d1


def test_sc_step_server_matches_launch_path(monkeypatch):
    """Three episodes (reset() with the block resident; the reference's host RandomState
    draws uploaded at each), an idle time-out mid-episode (the block exits by itself and the
    next post launches it again), stochastic lead times, the state rows after each episode."""
    srv, ref = _pair(monkeypatch, T=40, stochastic_leadtimes=True)
    rng = np.random.RandomState(5)
    launches0 = srv._server.launches
    for ep in range(3):
        assert np.array_equal(srv.reset(), ref.reset())
        done, t = False, 0
        while not done:
            if ep == 1 and t == 10:
                time.sleep(3 * srv._server.IDLE_US * 1e-6)
            done = _same(srv, ref, rng.uniform(-1, 1, srv.action_space.shape).astype(np.float32), (ep, t))
            t += 1
        assert np.array_equal(srv.stock, ref.stock), ep
        assert repr(srv.shipments()) == repr(ref.shipments()), ep
        with pytest.raises(IndexError):
            srv.step(np.zeros(srv.action_space.shape, dtype=np.float32))
    assert srv._server.launches - launches0 >= 2
    srv.close()
    srv.close()
    ref.close()


def test_sc_step_action_forms(monkeypatch):
    """step() takes the action as the reference does (:704, :716-717): any array-like of at
    least n_actions values, cast to float32, the rest unused; fewer raise IndexError. A list,
    a float64 array, a (1, A) array and a longer array step exactly as the float32 vector does
    (the facade's fast path), on the server and the launch path."""
    srv, ref = _pair(monkeypatch, T=12, seed=4)
    rng = np.random.RandomState(2)
    A = srv.action_space.shape[0]
    srv.reset()
    ref.reset()
    for t in range(12):
        a64 = rng.uniform(-1, 1, A + 3)
        forms = [a64[:A].tolist(), a64[:A], a64[:A].reshape(1, A), a64.astype(np.float32)]
        o1, r1, d1, _ = srv.step(forms[t % 4])
        o2, r2, d2, _ = ref.step(a64[:A].astype(np.float32))
        assert np.array_equal(o1, o2) and r1 == r2 and d1 == d2, t
        assert type(r1) is np.float64 and o1.dtype == np.float64
    for env in (srv, ref):
        env.reset()
        with pytest.raises(IndexError):
            env.step(np.zeros(A - 1, dtype=np.float32))
        env.close()


def test_sc_server_full_episode_and_terminal(monkeypatch):
    """A whole 360-step sc-2perstage episode (the terminal step's flags travel in the request)."""
    srv, ref = _pair(monkeypatch, T=360, seed=3)
    rng = np.random.RandomState(9)
    assert np.array_equal(srv.reset(), ref.reset())
    for t in range(360):
        done = _same(srv, ref, rng.uniform(-1, 1, srv.action_space.shape).astype(np.float32), t)
        assert done == (t == 359)
    srv.close()
    ref.close()


def test_sc_and_bg_servers_take_turns(monkeypatch):
    """A drop-in SupplyChainEnv and a drop-in BeerGameEnv stepped in turn, and two
    SupplyChainEnvs stepped in turn: at most one server is resident per device (each step of
    the other kind stops the resident one and launches its own), and every result is the
    launch path's."""
    from gym_supplychain_amd import BeerGameEnv
    from gym_supplychain_amd.envs import resident
    srv, ref = _pair(monkeypatch, T=20, seed=1)
    srv2, ref2 = _pair(monkeypatch, T=20, seed=2)
    monkeypatch.setenv("SCG_BG_SERVER", "1")
    bg = BeerGameEnv({})
    monkeypatch.setenv("SCG_BG_SERVER", "0")
    bg_ref = BeerGameEnv({})
    rng = np.random.RandomState(4)
    for e in (srv, ref, srv2, ref2):
        e.reset()
    bg.reset(), bg_ref.reset()
    for t in range(20):
        a = rng.uniform(-1, 1, srv.action_space.shape).astype(np.float32)
        _same(srv, ref, a, ("sc1", t))
        b = rng.randint(0, 10, 4)
        o1, r1, d1, _ = bg.step(b)
        o2, r2, d2, _ = bg_ref.step(b)
        assert np.array_equal(o1, o2) and r1 == r2 and d1 == d2, ("bg", t)
        _same(srv2, ref2, a, ("sc2", t))
        dev = srv._server._dev_index
        assert resident._RESIDENT.get(dev) is srv2._server
        assert srv._server.sv.running == 0 and bg._server.server.sv.running == 0
    for e in (srv, ref, srv2, ref2, bg, bg_ref):
        e.close()


def test_sc_block_gone_without_answering_is_relaunched(monkeypatch):
    """A block that exits while the host believes it runs (the mailbox's exit word raised
    behind the host's back) leaves the next request unanswered; the waiting step finds the
    stream idle at its next check and launches the block again, which serves the request."""
    srv, ref = _pair(monkeypatch, T=20, seed=8)
    sv = srv._server
    sv.sv.check_us = 5000
    srv.reset(), ref.reset()
    rng = np.random.RandomState(2)
    for t in range(20):
        if t in (4, 12):
            assert sv.sv.running == 1
            sv.box.exit_req = sv.box.exit_req + 1
            t0 = time.perf_counter()
            while sv.box.exit_seq != sv.box.exit_req and time.perf_counter() - t0 < 1.0:
                time.sleep(1e-4)
            assert sv.box.exit_seq == sv.box.exit_req
        _same(srv, ref, rng.uniform(-1, 1, srv.action_space.shape).astype(np.float32), t)
    assert sv.sv.relaunches == 2
    srv.close()
    ref.close()


def test_sc_device_synchronize_after_a_step_is_bounded(monkeypatch):
    """torch.cuda.synchronize() right after a step waits for the parked block's time-out
    (20 ms): within 25 ms."""
    srv, ref = _pair(monkeypatch, T=10, seed=6)
    srv.reset(), ref.reset()
    times = []
    for t in range(10):
        _same(srv, ref, np.zeros(srv.action_space.shape, dtype=np.float32), t)
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    assert max(times) < 25e-3, times
    srv.close()
    ref.close()


def test_sc_server_with_several_envs_through_the_c_abi():
    """scg_sc_server_step serves up to 64 envs: a 5-env sc-2perstage batch (node-parallel
    kernel, float64 observations) through the server, its actions read from device memory
    and its state kept in the block's LDS between steps, equals a twin stepped by vec.step(),
    over two episodes (the reset between them makes the block read the state again)."""
    import ctypes
    import gym_supplychain_amd as gsa
    from gym_supplychain_amd import _native as nat
    from gym_supplychain_amd.envs import resident
    N, T = 5, 12
    kw = dict(seed=4, device="cuda", kernel="nodes", obs_dtype=torch.float64, auto_reset=False, total_time_steps=T)
    a = gsa.make_vec("sc-2perstage-v0", N, **kw)
    b = gsa.make_vec("sc-2perstage-v0", N, **kw)
    A, O = a.n_actions, a.spec.n_obs
    act = torch.zeros((N, A), dtype=torch.float32, device="cuda")
    obs = torch.zeros((N, O), dtype=torch.float64, device="cuda")
    rew = torch.zeros((N,), dtype=torch.float64, device="cuda")
    stream, _ = resident.server_stream(torch.device("cuda"))
    box = nat.MappedBuffer(ctypes.sizeof(nat.ScServerBox))
    sv = nat.ScServer(box.host, box.dev, stream, act.data_ptr(), None, obs.data_ptr(), rew.data_ptr(), 20000, 0)
    done = ctypes.c_int32(0)
    gen = torch.Generator(device="cuda").manual_seed(8)
    try:
        for ep in range(2):
            assert torch.equal(a.reset(), b.reset())
            torch.cuda.synchronize()
            for t in range(T):
                x = torch.rand((N, A), generator=gen, device="cuda") * 2 - 1
                act.copy_(x)
                torch.cuda.synchronize()
                nat.check(nat.lib.scg_sc_server_step(ctypes.byref(a._cfg), ctypes.byref(a._st), ctypes.byref(sv),
                                                     ctypes.byref(done)))
                o, r, d, _ = b.step(x)
                assert torch.equal(obs, o) and torch.equal(rew, r), (ep, t)
                assert bool(done.value) == bool(d.all()), (ep, t)
            assert torch.equal(a.stock, b.stock), ep
    finally:
        nat.check(nat.lib.scg_sc_server_stop(ctypes.byref(sv)))
        resident.destroy_stream(stream)
