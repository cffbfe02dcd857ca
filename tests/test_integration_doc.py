"""INTEGRATION.md's reference-side binding, executed: the code a maintainer of the reference
would paste must match the library it binds (include/scgpu.h) and give the reference's
BeerGameEnv.step results (beergame_env.py:66-138).

The code blocks are read out of INTEGRATION.md itself, so the document cannot drift from
the ABI without this test failing.
"""
import os
import re

import numpy as np
import pytest

from conftest import REPO

DOC = os.path.join(REPO, "INTEGRATION.md")


def doc_block(tag):
    """The ```python block of INTEGRATION.md whose first line is `# [tag] ...`."""
    blocks = re.findall(r"```python\n(.*?)```", open(DOC).read(), flags=re.S)
    found = [b for b in blocks if b.startswith(f"# [{tag}]")]
    assert len(found) == 1, f"INTEGRATION.md must hold exactly one [{tag}] block"
    return found[0]


def run_binding(monkeypatch):
    from gym_supplychain_amd import _native as nat
    monkeypatch.setenv("SCGPU_LIB", nat.LIB_PATH)
    ns = {"__name__": "integration_doc"}
    exec(compile(doc_block("scgpu-binding"), "INTEGRATION.md[scgpu-binding]", "exec"), ns)
    return ns, nat


def test_binding_block_matches_the_library(monkeypatch):
    """The binding's own asserts (ABI version, all five struct sizes) pass, and each struct
    equals the package's binding field for field (names, offsets, sizes)."""
    import ctypes
    ns, nat = run_binding(monkeypatch)
    pairs = [("BgConfig", nat.BgConfig), ("BgState", nat.BgState), ("ScNode", nat.ScNode),
             ("ScConfig", nat.ScConfig), ("ScState", nat.ScState)]
    for name, ref in pairs:
        doc = ns[name]
        assert ctypes.sizeof(doc) == ctypes.sizeof(ref), name
        assert [f[0] for f in doc._fields_] == [f[0] for f in ref._fields_], name
        for f in ref._fields_:
            assert getattr(doc, f[0]).offset == getattr(ref, f[0]).offset, (name, f[0])
    bg = [ctypes.c_size_t() for _ in range(2)]
    nat.lib.scg_bg_struct_sizes(*map(ctypes.byref, bg))
    assert [v.value for v in bg] == [ctypes.sizeof(ns["BgConfig"]), ctypes.sizeof(ns["BgState"])]
    sc = [ctypes.c_size_t() for _ in range(3)]
    nat.lib.scg_sc_struct_sizes(*map(ctypes.byref, sc))
    assert [v.value for v in sc] == [ctypes.sizeof(ns[k]) for k in ("ScNode", "ScConfig", "ScState")]


def test_binding_block_prepares_the_default_game(monkeypatch):
    """The env block's host part: scg_bg_prepare through the documented structs (no GPU)."""
    import ctypes
    ns, _ = run_binding(monkeypatch)
    T = 35
    delays = (ctypes.c_int32 * (T + 1))(*([2] * (T + 1)))
    demand = (ctypes.c_int32 * T)(*([4] * 4 + [8] * 31))
    plan = (ctypes.c_int32 * (T + 1))()
    cfg = ns["BgConfig"](levels=4, max_weeks=T, inv_cost=1, backlog_cost=2, initial_shipment_value=4,
                         initial_orders_value=4, shipment_delays=ctypes.cast(delays, ctypes.c_void_p),
                         customer_demand=ctypes.cast(demand, ctypes.c_void_p), plan=ctypes.cast(plan, ctypes.c_void_p))
    assert ns["lib"].scg_bg_prepare(ctypes.byref(cfg)) == 0
    assert cfg.ring_slots == 3 and cfg.variant == 1


def env_block(n_envs):
    src = doc_block("beergame-env")
    line = "N, L, T = 65536, 4, 35"
    assert src.count(line) == 1
    return src.replace(line, f"N, L, T = {n_envs}, 4, 35")


@pytest.mark.gpu
def test_binding_blocks_run_the_reference_game(monkeypatch):
    """Both blocks, as documented, at N = 4,096 for a whole 35-week episode: every week's
    observation and reward equal the oracle's (pinned to the reference by the golden
    vectors), done at week 35, IndexError past the horizon (:79)."""
    import torch
    from oracle.beergame import DEFAULT_DEMAND, run_batch_episode
    ns, _ = run_binding(monkeypatch)
    N, L, T = 4096, 4, 35
    exec(compile(env_block(N), "INTEGRATION.md[beergame-env]", "exec"), ns)
    rng = np.random.RandomState(11)
    actions = rng.randint(-3, 9, size=(T, N, L))
    ref = run_batch_episode({}, np.tile(DEFAULT_DEMAND, (N, 1)), actions)
    obs = ns["reset"]()
    assert np.array_equal(obs.cpu().numpy(), ref["reset_obs"])
    acts = torch.as_tensor(actions, dtype=torch.int32, device="cuda")
    for w in range(T):
        obs, rew, done, info = ns["step"](acts[w])
        assert np.array_equal(obs.cpu().numpy(), ref["obs"][w]), w
        assert np.array_equal(rew.cpu().numpy(), ref["reward"][w]), w
        assert done == (w == T - 1) and info == {}
    bufs = ns["bufs"]
    assert np.array_equal(bufs["inventory_costs"].cpu().numpy(), ref["inventory_costs"])
    assert np.array_equal(bufs["backlog_costs"].cpu().numpy(), ref["backlog_costs"])
    with pytest.raises(IndexError):
        ns["step"](acts[0])
    ns["reset"]()                          # a second episode through the same binding
    obs, rew, _, _ = ns["step"](acts[0])
    assert np.array_equal(rew.cpu().numpy(), ref["reward"][0])
