"""C ABI checks that need no GPU: exports, struct layout, host-side config logic."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "scgpu.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"SCG_API\s+[\w\s\*]+?\b(scg_\w+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert {"scg_bg_prepare", "scg_bg_reset", "scg_bg_step", "scg_bg_rollout", "scg_poisson_table",
            "scg_last_error", "scg_abi_version"} <= set(syms)


def test_library_exports_every_declared_symbol():
    from gym_supplychain_amd import _native as nat
    out = subprocess.run(["nm", "-D", "--defined-only", nat.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (scg_\w+)", out))
    assert set(declared_symbols()) == exported
    assert set(declared_symbols()) == set(nat.SIGNATURES)
    for s in declared_symbols():
        getattr(nat.lib, s)


def test_struct_layout_matches_ctypes():
    from gym_supplychain_amd import _native as nat
    cs, ss = ctypes.c_size_t(), ctypes.c_size_t()
    assert nat.lib.scg_bg_struct_sizes(ctypes.byref(cs), ctypes.byref(ss)) == 0
    assert cs.value == ctypes.sizeof(nat.BgConfig) and ss.value == ctypes.sizeof(nat.BgState)


def test_poisson_table_matches_oracle():
    from gym_supplychain_amd import _native as nat
    from oracle.poisson import poisson_thresholds
    for lam in [0.0, 0.25, 1.0, 3.0, 4.5, 8.0, 12.0, 33.3, 100.0]:
        assert nat.poisson_table(lam) == poisson_thresholds(lam).tolist()
    with pytest.raises(ValueError):
        nat.poisson_table(-2.0)
    with pytest.raises(ValueError):
        nat.poisson_table(float("nan"))


def _plan(delays, T, demand=None):
    """Run scg_bg_prepare on a shipment_delays list ([d0] + per-week), return the plan."""
    from gym_supplychain_amd import _native as nat
    c = nat.BgConfig()
    c.levels, c.max_weeks = 4, T
    d = (ctypes.c_int32 * (T + 1))(*delays)
    dem = (ctypes.c_int32 * T)(*(demand or [8] * T))
    plan = (ctypes.c_int32 * (T + 1))()
    c.shipment_delays = ctypes.cast(d, ctypes.c_void_p)
    c.customer_demand = ctypes.cast(dem, ctypes.c_void_p)
    c.plan = ctypes.cast(plan, ctypes.c_void_p)
    rc = nat.lib.scg_bg_prepare(ctypes.byref(c))
    return rc, list(plan), c.ring_slots


def _expected_plan(delays, T):
    """Independent re-derivation from the absolute-week table of beergame_env.py:46-52."""
    writes = {t: 1 for t in range(1, min(delays[0], T) + 1)}
    plan = [0]
    for w in range(1, T + 1):
        arrive = w in writes
        d = delays[w]
        if d == 0:
            mode = 0
        elif w + d > T:
            mode = 3
        elif (w + d) in writes:
            mode = 2
        else:
            mode = 1
            writes[w + d] = 1
        plan.append(mode | (4 if arrive else 0) | (d << 8))
    return plan


@pytest.mark.parametrize("seed", range(8))
def test_prepare_plan(seed):
    rng = np.random.RandomState(seed)
    T = int(rng.randint(1, 60))
    delays = [2] + rng.randint(0, 1 + int(rng.randint(1, 10)), size=T).tolist()
    rc, plan, R = _plan(delays, T)
    assert rc == 0
    assert plan == _expected_plan(delays, T)
    assert R == max(delays) + 1


def test_prepare_rejects_bad_configs():
    from gym_supplychain_amd import _native as nat
    rc, _, _ = _plan([2] + [-1] * 5, 5)
    assert rc == nat.SCG_ERR_INVALID and "shipment_delays" in nat.last_error()
    rc, _, _ = _plan([2] + [nat.BG_MAX_DELAY + 1] * 5, 5)
    assert rc == nat.SCG_ERR_INVALID


def test_config_mirrors_reference_defaults_and_errors():
    from gym_supplychain_amd.envs import BeerGameConfig
    c = BeerGameConfig({})
    assert (c.levels, c.max_weeks, c.inv_cost, c.backlog_cost) == (4, 35, 1, 2)
    assert c.customer_demand.tolist() == [4] * 4 + [8] * 31
    assert c.initial_inventory.tolist() == [12] * 4
    assert c.shipment_delays.tolist() == [2] * 36
    c = BeerGameConfig({"customer_demand": [1, 2, 3], "initial_inventory": [1.9, 2, 3, 4]})
    assert c.max_weeks == 3 and c.initial_inventory.tolist() == [1, 2, 3, 4]
    with pytest.raises(IndexError):  # table sizing reads shipment_delays[0..T] (:47-48)
        BeerGameConfig({"shipment_delays": [2, 2]})
    with pytest.raises(TypeError):   # float costs break the int ledgers (:131)
        BeerGameConfig({"inv_cost": 1.5})
    with pytest.raises(ValueError):
        BeerGameConfig({"levels": 6})  # default initial_inventory has 4 entries


def test_step_rejects_shards_beyond_int32_before_any_launch():
    """The step kernel takes the shard's env count as one preloaded 32-bit argument: the
    launcher rejects larger shards (validation runs before any HIP call, so no GPU needed)."""
    from gym_supplychain_amd import _native as nat
    T = 35
    c = nat.BgConfig()
    c.levels, c.max_weeks = 4, T
    d = (ctypes.c_int32 * (T + 1))(*([2] * (T + 1)))
    dem = (ctypes.c_int32 * T)(*([8] * T))
    plan = (ctypes.c_int32 * (T + 1))()
    c.shipment_delays = ctypes.cast(d, ctypes.c_void_p)
    c.customer_demand = ctypes.cast(dem, ctypes.c_void_p)
    c.plan = ctypes.cast(plan, ctypes.c_void_p)
    assert nat.lib.scg_bg_prepare(ctypes.byref(c)) == 0
    st = nat.BgState()
    st.n_envs, st.env_offset, st.week = 2 ** 31, 0, 0
    fake = ctypes.c_void_p(0x1000)  # never dereferenced: the call fails validation first
    for f in ("inventory", "backlog", "orders_placed", "shipments"):
        setattr(st, f, fake)
    out = ctypes.c_int32(0)
    rc = nat.lib.scg_bg_step(ctypes.byref(c), ctypes.byref(st), fake, fake, fake, None, 0, ctypes.byref(out), None)
    assert rc == nat.SCG_ERR_INVALID and "n_envs" in nat.last_error()


def test_step_server_validates_before_any_launch():
    """scg_bg_server_attach / _post / _detach / _stop: every argument the resident wave depends
    on is checked on the host before anything is launched (a slot without buffers, the null
    stream, levels or an idle time-out out of range, all slots taken; more than 64 envs, a
    config that is not the server's, BeerGameEnv2, the slab layout, a step before reset or past
    the horizon, a detached slot); attach and detach keep the polled slot count; stopping a
    server that never ran is a no-op."""
    from gym_supplychain_amd import _native as nat
    T = 35
    c = nat.BgConfig()
    c.levels, c.max_weeks = 4, T
    d = (ctypes.c_int32 * (T + 1))(*([2] * (T + 1)))
    dem = (ctypes.c_int32 * T)(*([8] * T))
    plan = (ctypes.c_int32 * (T + 1))()
    c.shipment_delays = ctypes.cast(d, ctypes.c_void_p)
    c.customer_demand = ctypes.cast(dem, ctypes.c_void_p)
    c.plan = ctypes.cast(plan, ctypes.c_void_p)
    assert nat.lib.scg_bg_prepare(ctypes.byref(c)) == 0
    fake = 0x1000  # never dereferenced: every call below fails validation first
    st = nat.BgState()
    st.n_envs, st.env_offset, st.week = 1, 0, 0
    for f in ("inventory", "backlog", "orders_placed", "shipments"):
        setattr(st, f, fake)
    box = nat.BgServerBox()  # ordinary host memory: attach/detach only write the mailbox
    sv = nat.BgServer(ctypes.addressof(box), fake, fake, 4, nat.SCG_DEMAND_FIXED, 20000, 0)
    done = ctypes.c_int32(0)

    def attach(slot, expect=0, text=""):
        rc = nat.lib.scg_bg_server_attach(ctypes.byref(sv), ctypes.byref(slot))
        assert rc == expect and text in (nat.last_error() if rc else ""), (rc, nat.last_error())

    slot = nat.BgServerSlot(None, fake, None, None, fake, -1)
    attach(slot, nat.SCG_ERR_INVALID, "required")
    slot.obs = fake
    sv.stream = None
    attach(slot, nat.SCG_ERR_INVALID, "null stream")
    sv.stream = fake
    sv.idle_us = 10
    attach(slot, nat.SCG_ERR_INVALID, "idle_us")
    sv.idle_us = 20000
    sv.levels = 17
    attach(slot, nat.SCG_ERR_INVALID, "levels")
    sv.levels = 4
    slots = [nat.BgServerSlot(None, fake, None, fake, fake, -1) for _ in range(nat.BG_SERVER_SLOTS)]
    for k, s in enumerate(slots):
        attach(s)
        assert s.index == k and box.n_slots == k + 1
    attach(slot, nat.SCG_ERR_INVALID, "slots are taken")
    for k in (3, nat.BG_SERVER_SLOTS - 1):
        assert nat.lib.scg_bg_server_detach(ctypes.byref(slots[k])) == 0 and slots[k].index == -1
    assert box.n_slots == nat.BG_SERVER_SLOTS - 1 and sv.slots_used == (1 << nat.BG_SERVER_SLOTS) - 1 - 8 - (1 << 14)
    attach(slot)
    assert slot.index == 3  # the lowest free slot
    slot = slots[0]

    def post(expect, text):
        rc = nat.lib.scg_bg_server_post(ctypes.byref(c), ctypes.byref(st), ctypes.byref(slot))
        assert rc == expect and text in nat.last_error(), (rc, nat.last_error())

    st.n_envs = 65
    post(nat.SCG_ERR_INVALID, "64")
    st.n_envs = 1
    st.slab = fake
    post(nat.SCG_ERR_INVALID, "slab")
    st.slab = None
    st.week = -1
    post(nat.SCG_ERR_NOT_RESET, "reset")
    st.week = T
    post(nat.SCG_ERR_PAST_HORIZON, "terminal")
    st.week = 0
    c.demand_mode = nat.SCG_DEMAND_UNIFORM
    c.demand_lo, c.demand_hi = 0, 8
    post(nat.SCG_ERR_INVALID, "not the server's")
    c.demand_mode = nat.SCG_DEMAND_FIXED
    c.variant = 2
    post(nat.SCG_ERR_INVALID, "variant 1")
    c.variant = 1
    assert nat.lib.scg_bg_server_detach(ctypes.byref(slot)) == 0
    post(nat.SCG_ERR_INVALID, "not attached")
    rc = nat.lib.scg_bg_server_wait(ctypes.byref(st), ctypes.byref(slot), 0, ctypes.byref(done))
    assert rc == nat.SCG_ERR_INVALID
    # nothing was posted or launched
    assert sv.running == 0 and sv.launches == 0 and all(box.req[k].req_seq == 0 for k in range(16))
    assert nat.lib.scg_bg_server_stop(ctypes.byref(sv)) == 0
    assert nat.lib.scg_bg_server_stop(None) == nat.SCG_ERR_INVALID


def test_step_server_check_word_mixes_every_word():
    """The request line's check (scg_bg_server_line_check, recomputed by the wave) is a mixing
    hash: a read that mixes two requests is caught even when two action words move by amounts
    a weighted sum would cancel (+19k in word 8, -17k in word 9), and when any single word
    changes."""
    from gym_supplychain_amd import _native as nat
    rng = np.random.default_rng(0)
    line = nat.BgServerLine()
    for k in range(200):
        words = rng.integers(0, 2 ** 32, 16, dtype=np.uint64)
        ctypes.memmove(ctypes.addressof(line), words.astype(np.uint32).tobytes(), 64)
        h = nat.lib.scg_bg_server_line_check(ctypes.byref(line))
        w2 = words.astype(np.uint32).copy()
        w2[8] = np.uint32((int(w2[8]) + 19 * (k + 1)) % 2 ** 32)
        w2[9] = np.uint32((int(w2[9]) - 17 * (k + 1)) % 2 ** 32)
        ctypes.memmove(ctypes.addressof(line), w2.tobytes(), 64)
        assert nat.lib.scg_bg_server_line_check(ctypes.byref(line)) != h
        for i in (0, 1, 2, 3, 4, 5, 6, 8 + k % 8):
            w3 = words.astype(np.uint32).copy()
            w3[i] ^= np.uint32(1 << (k % 32))
            ctypes.memmove(ctypes.addressof(line), w3.tobytes(), 64)
            assert nat.lib.scg_bg_server_line_check(ctypes.byref(line)) != h
        w4 = words.astype(np.uint32).copy()
        w4[7] ^= np.uint32(0xFFFFFFFF)  # the check word itself is not hashed
        ctypes.memmove(ctypes.addressof(line), w4.tobytes(), 64)
        assert nat.lib.scg_bg_server_line_check(ctypes.byref(line)) == h


def test_uniform_ints_rejects_env_ids_and_sizes_before_any_launch():
    """scg_uniform_ints: the Philox env counter is 32-bit and the per-env word count int32, so
    ids past 2^32 and rows*width past INT32_MAX are rejected before any HIP call."""
    from gym_supplychain_amd import _native as nat
    fake = ctypes.c_void_p(0x1000)  # never dereferenced
    rc = nat.lib.scg_uniform_ints(1, 2 ** 32 - 4, 8, 1, 4, 0, 0, 9, fake, None)
    assert rc == nat.SCG_ERR_INVALID and "2^32" in nat.last_error()
    rc = nat.lib.scg_uniform_ints(1, -1, 8, 1, 4, 0, 0, 9, fake, None)
    assert rc == nat.SCG_ERR_INVALID
    rc = nat.lib.scg_uniform_ints(1, 0, 8, 65536, 65536, 0, 0, 9, fake, None)
    assert rc == nat.SCG_ERR_INVALID and "int32" in nat.last_error()


def test_slab_layout():
    """scg_bg_slab_layout: 16-byte header, six [N][L] rows, the ring, two int64 returns,
    the optional history; rejects batches whose rows would not stay 16-byte aligned."""
    import ctypes
    from gym_supplychain_amd import _native as nat
    T = 35
    c = nat.BgConfig()
    c.levels, c.max_weeks = 4, T
    d = (ctypes.c_int32 * (T + 1))(*([2] * (T + 1)))
    dem = (ctypes.c_int32 * T)(*([8] * T))
    plan = (ctypes.c_int32 * (T + 1))()
    c.shipment_delays, c.customer_demand = ctypes.cast(d, ctypes.c_void_p), ctypes.cast(dem, ctypes.c_void_p)
    c.plan = ctypes.cast(plan, ctypes.c_void_p)
    assert nat.lib.scg_bg_prepare(ctypes.byref(c)) == 0
    N, L, R = 65536, 4, c.ring_slots
    assert R == 3
    off = (ctypes.c_int64 * nat.SLAB_FIELDS)()
    assert nat.lib.scg_bg_slab_layout(ctypes.byref(c), N, 1, off) == 0
    NL = N * L
    assert off[nat.SLAB_ERROR] == 0 and off[nat.SLAB_INVENTORY] == 4
    assert [off[nat.SLAB_INVENTORY + f] for f in range(6)] == [4 + f * NL for f in range(6)]
    assert off[nat.SLAB_RING] == 4 + 6 * NL
    assert off[nat.SLAB_EPISODE_RETURN] == 4 + (6 + R) * NL and off[nat.SLAB_EPISODE_RETURN] % 2 == 0
    assert off[nat.SLAB_FINAL_RETURN] == off[nat.SLAB_EPISODE_RETURN] + 2 * N
    assert off[nat.SLAB_HISTORY] == off[nat.SLAB_FINAL_RETURN] + 2 * N
    assert off[nat.SLAB_TOTAL] == off[nat.SLAB_HISTORY] + (T + 1) * NL
    assert nat.lib.scg_bg_slab_layout(ctypes.byref(c), N, 0, off) == 0
    assert off[nat.SLAB_TOTAL] == off[nat.SLAB_HISTORY]
    assert nat.lib.scg_bg_slab_layout(ctypes.byref(c), 77, 0, off) == 0                     # 77 * 4 % 4 == 0
    c.levels = 3
    assert nat.lib.scg_bg_slab_layout(ctypes.byref(c), 77, 0, off) == nat.SCG_ERR_INVALID


def _prepare_full(delays, T, variant=1):
    from gym_supplychain_amd import _native as nat
    c = nat.BgConfig()
    c.levels, c.max_weeks, c.full_table, c.variant = 4, T, 1, variant
    d = (ctypes.c_int32 * (T + 1))(*delays)
    dem = (ctypes.c_int32 * T)(*([8] * T))
    plan = (ctypes.c_int32 * (T + 1))()
    c.shipment_delays, c.customer_demand = ctypes.cast(d, ctypes.c_void_p), ctypes.cast(dem, ctypes.c_void_p)
    c.plan = ctypes.cast(plan, ctypes.c_void_p)
    return nat.lib.scg_bg_prepare(ctypes.byref(c)), list(plan), c.ring_slots


@pytest.mark.parametrize("seed", range(6))
def test_prepare_full_table(seed):
    """full_table: R = the reference's row count max(T+1, max_w(w+d_w+1)) + 1
    (beergame_env.py:46-50), slot s = week s, and the weeks that ship past the horizon are
    stored (STORE/ADD into rows > T) instead of dropped."""
    from oracle.beergame import shipment_rows
    rng = np.random.RandomState(100 + seed)
    T = int(rng.randint(1, 40))
    delays = [2] + rng.randint(0, 1 + int(rng.randint(1, 9)), size=T).tolist()
    rc, plan, R = _prepare_full(delays, T)
    assert rc == 0 and R == shipment_rows(T, np.asarray(delays))
    written = set(range(1, delays[0] + 1))   # the initial pipeline, even past T (:52)
    for w in range(1, T + 1):
        d = delays[w]
        mode = plan[w] & 3
        assert plan[w] >> 8 == d and bool(plan[w] & 4) == (w in written)
        if d == 0:
            assert mode == 0
        else:
            assert mode == (2 if w + d in written else 1), (w, d)
            written.add(w + d)


def test_prepare_full_table_limits():
    from gym_supplychain_amd import _native as nat
    rc, _, R = _prepare_full([2] * 130, 129)             # 133 rows: past the slab's 127, any table is kept
    assert rc == 0 and R == 133
    rc, _, R = _prepare_full([2] + [70] * 150, 150)      # a 150-week horizon with delay 70: 222 rows
    assert rc == 0 and R == 222
    rc, _, _ = _prepare_full([2] + [nat.BG_MAX_DELAY + 1] * 3, 3)
    assert rc == nat.SCG_ERR_INVALID and "shipment_delays" in nat.last_error()
    rc, _, _ = _prepare_full([2] * 36, 35, variant=2)
    assert rc == nat.SCG_ERR_INVALID and "full_table" in nat.last_error()


def test_server_struct_layouts_match_the_library():
    """The step servers' structs as ctypes lays them out are the sizes the library asserts at
    compile time (scg_beergame.hip, scg_supplychain.hip static_asserts), so a binding that
    drifted from include/scgpu.h fails here rather than on the GPU."""
    from gym_supplychain_amd import _native as nat
    assert ctypes.sizeof(nat.BgServerLine) == 64
    assert ctypes.sizeof(nat.BgServerBox) == 17 * 64 + 64 + nat.BG_SERVER_SLOTS * nat.BG_SERVER_ARGS_BYTES
    assert nat.BgServerBox.done_seq.offset == 16 * 64 and nat.BgServerBox.args.offset == 18 * 64
    assert ctypes.sizeof(nat.BgServer) == 72 and ctypes.sizeof(nat.BgServerSlot) == 64
    assert ctypes.sizeof(nat.ScServerBox) == 192 and nat.ScServerBox.action.offset == 64
    assert nat.ScServerBox.done_seq.offset == 128 and ctypes.sizeof(nat.ScServer) == 104
