"""GPU tests of the drop-in BeerGameEnv's step server (include/scgpu.h scg_bg_server_*: one
resident wave per device and level count serving every drop-in env of the process from a
host-mapped mailbox) in the ways a trainer uses it: one env over several episodes, several
envs stepped in turn (an SB3 DummyVecEnv), beside a BeerGameVecEnv on torch's stream, beside
kernels on other streams, a device-wide synchronize right after a step, a wave gone without
answering, and envs stepped from several threads. Every result is compared, bit for bit,
with the launch path (SCG_BG_SERVER=0: one step-kernel launch and one synchronisation per
step), which the golden tests of test_gpu_beergame.py pin to the reference."""
import threading
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _info(levels, T, seed):
    rng = np.random.RandomState(seed)
    return dict(levels=levels, initial_inventory=[12] * levels, customer_demand=rng.randint(0, 12, T).tolist(),
                shipment_delays=rng.randint(0, 4, T).tolist())


def _pair(info, monkeypatch):
    from gym_supplychain_amd import BeerGameEnv
    monkeypatch.setenv("SCG_BG_SERVER", "1")
    srv = BeerGameEnv(info)
    monkeypatch.setenv("SCG_BG_SERVER", "0")
    ref = BeerGameEnv(info)
    assert srv._server is not None and ref._server is None
    return srv, ref


def _same(srv, ref, a, where):
    o1, r1, d1, _ = srv.step(a)
    o2, r2, d2, _ = ref.step(a)
    assert np.array_equal(o1, o2) and r1 == r2 and d1 == d2, where
    assert srv.week == ref.week, where


def _same_state(srv, ref, where):
    for attr in ("inventory", "backlog", "orders_placed", "inventory_costs", "backlog_costs", "all_orders_placed",
                 "shipments"):
        assert np.array_equal(getattr(srv, attr), getattr(ref, attr)), (where, attr)


@pytest.mark.parametrize("levels", [4, 10])
def test_step_server_matches_launch_path(levels, monkeypatch):
    """One env against the launch path, week for week: observation, reward, done and the state
    rows, over three episodes (reset() leaves the shared wave running), an idle time-out
    mid-episode (the wave exits by itself and the next post launches it again), and L = 10 > 8
    (the action row read from host-mapped memory instead of travelling in the request line)."""
    T = 30
    rng = np.random.RandomState(levels)
    srv, ref = _pair(_info(levels, T, levels), monkeypatch)
    launches0 = srv._server.server.launches
    for ep in range(3):
        assert np.array_equal(srv.reset(), ref.reset())
        for w in range(T):
            if ep == 1 and w == 10:
                time.sleep(3 * srv._server.server.IDLE_US * 1e-6)  # the wave times out and exits
            _same(srv, ref, rng.randint(-3, 15, levels), (ep, w))
        _same_state(srv, ref, ep)
        with pytest.raises(IndexError):
            srv.step(np.zeros(levels, dtype=np.int64))
    assert srv._server.server.launches - launches0 >= 2  # the first post, and one after the time-out
    srv.close()
    srv.close()  # idempotent
    ref.close()


def test_eight_dropin_envs_share_one_wave(monkeypatch):
    """8 drop-in envs stepped round-robin over two episodes each, as SB3's DummyVecEnv does:
    every result equals its launch-path twin, all 8 hold slots of ONE server (one resident
    wave, one stream), and the wave is launched once for all of them."""
    T, L = 24, 4
    pairs = [_pair(_info(L, T, 100 + k), monkeypatch) for k in range(8)]
    servers = {id(s._server.server) for s, _ in pairs}
    assert len(servers) == 1
    assert len({s._server.slot.index for s, _ in pairs}) == 8
    server = pairs[0][0]._server.server
    server.stop()
    launches0 = server.launches
    rng = np.random.RandomState(7)
    for ep in range(2):
        for s, r in pairs:
            assert np.array_equal(s.reset(), r.reset())
        for w in range(T):
            for k, (s, r) in enumerate(pairs):
                _same(s, r, rng.randint(0, 15, L), (ep, w, k))
        for k, (s, r) in enumerate(pairs):
            _same_state(s, r, (ep, k))
    assert server.launches - launches0 == 1
    for s, r in pairs:
        s.close()
        r.close()


def test_more_envs_than_slots_start_a_second_server(monkeypatch):
    """Past BG_SERVER_SLOTS drop-in envs of one level count on one device a second server
    (its own wave) takes the rest; a closed env's slot is reused by the next env."""
    from gym_supplychain_amd import _native as nat
    T, L = 12, 4
    n = nat.BG_SERVER_SLOTS + 2
    pairs = [_pair(_info(L, T, 200 + k), monkeypatch) for k in range(n)]
    servers = {id(s._server.server) for s, _ in pairs}
    assert len(servers) == 2
    rng = np.random.RandomState(3)
    for s, r in pairs:
        assert np.array_equal(s.reset(), r.reset())
    for w in range(T):
        for k, (s, r) in enumerate(pairs):
            _same(s, r, rng.randint(0, 15, L), (w, k))
    idx = pairs[5][0]._server.slot.index
    first = pairs[5][0]._server.server
    pairs[5][0].close()
    s, r = _pair(_info(L, T, 999), monkeypatch)
    assert s._server.server is first and s._server.slot.index == idx
    assert np.array_equal(s.reset(), r.reset())
    for w in range(T):
        _same(s, r, rng.randint(0, 15, L), w)
    for s2, r2 in pairs + [(s, r)]:
        s2.close()
        r2.close()


def test_dropin_env_beside_vec_env_on_torch_stream(monkeypatch):
    """A drop-in env stepping between the steps of a BeerGameVecEnv on torch's current stream:
    both give what each gives alone (the vec env against a twin stepped with no server around,
    the drop-in env against its launch-path twin)."""
    from gym_supplychain_amd import BeerGameVecEnv
    T, L, N = 20, 4, 4096
    info = _info(L, T, 5)
    srv, ref = _pair(info, monkeypatch)
    vec = BeerGameVecEnv(N, info, demand="fixed", device="cuda", auto_reset=False)
    gen = torch.Generator(device="cuda").manual_seed(0)
    acts = torch.randint(0, 15, (T, N, L), generator=gen, device="cuda", dtype=torch.int32)
    srv.reset(), ref.reset(), vec.reset()
    rng = np.random.RandomState(11)
    got = []
    for w in range(T):
        o, r, d, _ = vec.step(acts[w])  # enqueued on torch's stream, not waited for
        _same(srv, ref, rng.randint(0, 15, L), w)
        got.append((o.clone(), r.clone()))
    torch.cuda.synchronize()
    srv.close()
    alone = BeerGameVecEnv(N, info, demand="fixed", device="cuda", auto_reset=False)
    alone.reset()
    for w in range(T):
        o, r, d, _ = alone.step(acts[w])
        assert torch.equal(o, got[w][0]) and torch.equal(r, got[w][1]), w
    ref.close()


def test_parked_wave_does_not_hold_other_streams(monkeypatch):
    """While the wave waits for the next request (up to its 20 ms idle time-out), kernels on
    eight other streams of the process — more than the 4 hardware queues a priority class
    has (GPU_MAX_HW_QUEUES) — complete in well under that time: the server's stream is of the
    highest priority, so no normal-priority stream shares its hardware queue."""
    T, L = 8, 4
    srv, ref = _pair(_info(L, T, 9), monkeypatch)
    srv.reset(), ref.reset()
    streams = [torch.cuda.Stream() for _ in range(8)]
    x = torch.ones(1 << 16, device="cuda")
    for s in streams:  # warm each stream up (first use)
        with torch.cuda.stream(s):
            x.add(1)
        s.synchronize()
    worst = 0.0
    for w in range(T):
        _same(srv, ref, np.full(L, 5), w)  # the wave is resident and parked after this
        for s in streams:
            t0 = time.perf_counter()
            with torch.cuda.stream(s):
                x.add(1)
            s.synchronize()
            worst = max(worst, time.perf_counter() - t0)
    assert worst < 5e-3, f"a kernel on another stream took {worst * 1e3:.2f} ms beside the parked wave"
    srv.close()
    ref.close()


def test_device_synchronize_right_after_a_step_is_bounded(monkeypatch):
    """torch.cuda.synchronize() right after a step waits for the parked wave to time out
    (IDLE_US = 20 ms): it returns within 25 ms, and the next step launches the wave again."""
    T, L = 10, 4
    srv, ref = _pair(_info(L, T, 13), monkeypatch)
    srv.reset(), ref.reset()
    times = []
    for w in range(T):
        _same(srv, ref, np.full(L, w % 7), w)
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    assert max(times) < 25e-3, times
    srv.close()
    ref.close()


def test_wave_gone_without_answering_is_relaunched(monkeypatch):
    """A wave that exits while the host believes it runs (forced here by raising the mailbox's
    exit word behind the host's back) leaves the next request unanswered; the waiting step
    finds the wave's stream idle at its next check, launches the wave again — which serves the
    pending request first — and the result is the launch path's."""
    T, L = 12, 4
    srv, ref = _pair(_info(L, T, 17), monkeypatch)
    slot = srv._server
    server = slot.server
    server.sv.check_us = 5000
    srv.reset(), ref.reset()
    for w in range(T):
        if w in (3, 8):
            assert server.sv.running == 1
            server.box.exit_req = server.box.exit_req + 1  # the wave exits; the host is not told
            t0 = time.perf_counter()
            while server.box.exit_seq != server.box.exit_req and time.perf_counter() - t0 < 1.0:
                time.sleep(1e-4)
            assert server.box.exit_seq == server.box.exit_req
        _same(srv, ref, np.full(L, 3 + w % 5), w)
    assert slot.slot.relaunches == 2
    server.sv.check_us = 0
    srv.close()
    ref.close()


def test_dropin_envs_stepped_from_threads(monkeypatch):
    """Four threads each stepping two drop-in envs of the shared server (the GIL is released
    while a step waits): every trajectory equals its launch-path twin stepped afterwards."""
    T, L = 20, 4
    from gym_supplychain_amd import BeerGameEnv
    monkeypatch.setenv("SCG_BG_SERVER", "1")
    infos = [_info(L, T, 300 + k) for k in range(8)]
    envs = [BeerGameEnv(i) for i in infos]
    acts = np.random.RandomState(1).randint(0, 15, (8, T, L))
    out = [[] for _ in range(8)]
    errors = []

    def run(ks):
        try:
            for k in ks:
                out[k].append(envs[k].reset())
            for w in range(T):
                for k in ks:
                    o, r, d, _ = envs[k].step(acts[k, w])
                    out[k].append((o, r, d))
        except Exception as exc:  # pragma: no cover - reported below
            errors.append(exc)

    threads = [threading.Thread(target=run, args=((2 * j, 2 * j + 1),)) for j in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    assert not errors, errors
    monkeypatch.setenv("SCG_BG_SERVER", "0")
    for k in range(8):
        ref = BeerGameEnv(infos[k])
        assert np.array_equal(out[k][0], ref.reset())
        for w in range(T):
            o, r, d, _ = ref.step(acts[k, w])
            o1, r1, d1 = out[k][1 + w]
            assert np.array_equal(o, o1) and r == r1 and d == d1, (k, w)
        ref.close()
        envs[k].close()


def test_server_slot_with_several_envs_through_the_c_abi():
    """A slot serves up to 64 envs (include/scgpu.h scg_bg_server_*): a 5-env BeerGameVecEnv
    (separate state buffers) stepped through scg_bg_server_step, its action row read from
    device memory (no inline row), equals a twin stepped by vec.step(), week for week."""
    import ctypes
    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd import _native as nat
    from gym_supplychain_amd.envs import resident
    T, L, N = 20, 4, 5
    info = _info(L, T, 21)
    a = BeerGameVecEnv(N, info, demand="fixed", device="cuda", auto_reset=False, state_slab=False)
    b = BeerGameVecEnv(N, info, demand="fixed", device="cuda", auto_reset=False, state_slab=False)
    act = torch.zeros((N, L), dtype=torch.int32, device="cuda")
    obs = torch.zeros((N, L), dtype=torch.int32, device="cuda")
    rew = torch.zeros((N,), dtype=torch.int32, device="cuda")
    stream, _ = resident.server_stream(torch.device("cuda"))
    box = nat.MappedBuffer(ctypes.sizeof(nat.BgServerBox))
    sv = nat.BgServer(box.host, box.dev, stream, L, nat.SCG_DEMAND_FIXED, 20000, 0)
    slot = nat.BgServerSlot(None, act.data_ptr(), None, obs.data_ptr(), rew.data_ptr(), -1)
    nat.check(nat.lib.scg_bg_server_attach(ctypes.byref(sv), ctypes.byref(slot)))
    done = ctypes.c_int32(0)
    try:
        assert torch.equal(a.reset(), b.reset())
        torch.cuda.synchronize()
        gen = torch.Generator(device="cuda").manual_seed(3)
        for w in range(T):
            x = torch.randint(0, 15, (N, L), generator=gen, device="cuda", dtype=torch.int32)
            act.copy_(x)
            torch.cuda.synchronize()  # the row is in place before the post
            nat.check(nat.lib.scg_bg_server_step(ctypes.byref(a._cfg), ctypes.byref(a._st), ctypes.byref(slot),
                                                 ctypes.byref(done)))
            o, r, d, _ = b.step(x)
            assert torch.equal(obs, o) and torch.equal(rew, r), w
            assert bool(done.value) == bool(d.all()) and a.week == b.week == w + 1
        assert torch.equal(a.inventory, b.inventory) and torch.equal(a.backlog, b.backlog)
    finally:
        nat.check(nat.lib.scg_bg_server_detach(ctypes.byref(slot)))
        nat.check(nat.lib.scg_bg_server_stop(ctypes.byref(sv)))
        resident.destroy_stream(stream)
