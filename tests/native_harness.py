"""Builds tests/native/sc_host_harness.cpp (test-only host build of the SupplyChain kernel
body) with hipcc and binds it with ctypes. Used by tests/test_sc_host.py."""
import ctypes
import os
import subprocess

import numpy as np

from conftest import PKG_ROOT, REPO

SRC = os.path.join(REPO, "tests", "native", "sc_host_harness.cpp")
OUT = os.path.join(REPO, "tests", "native", "_build", "libsc_host.so")
CSRC = os.path.join(PKG_ROOT, "csrc")


def build(defines=()):
    """The harness library; `defines` (e.g. ("SCG_STAGED_SHIP_BITS=1",)) build a variant of its own."""
    out = OUT if not defines else OUT.replace(".so", "_" + "_".join(d.replace("=", "") for d in defines) + ".so")
    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
        [os.path.join(REPO, "include", "scgpu.h")]
    if not (os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps)):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        tmp = f"{out}.{os.getpid()}.tmp"  # concurrent test workers: build aside, rename into place
        subprocess.run(["hipcc", "-std=c++17", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-Wno-pass-failed",
                        "--offload-arch=gfx950", "-I", os.path.join(REPO, "include"), "-I", CSRC] +
                       [f"-D{d}" for d in defines] + ["-o", tmp, SRC], check=True)
        os.replace(tmp, out)
    lib = ctypes.CDLL(out)
    lib.sch_episode.restype = ctypes.c_int
    lib.sch_episode_level.restype = ctypes.c_int
    lib.sch_episode_ledger.restype = ctypes.c_int
    lib.sch_episode_staged.restype = ctypes.c_int
    lib.sch_episode_nodes.restype = ctypes.c_int
    lib.sch_nodes_fallbacks.restype = ctypes.c_int
    lib.sch_episode_nodes_serial.restype = ctypes.c_int
    lib.sch_episode_nodes_ledger.restype = ctypes.c_int
    return lib


def run_episode(lib, cfg, nodes, lt_thr, seed, env_id, episode, actions, level=False, ledger=False, staged=False,
                nodes_kernel=False, nodes_serial=False):
    """Reset + len(actions) steps of one env; returns obs [T+1, O], rewards [T],
    stock [T+1, NP], heaps (tk, val, size) per snapshot; with ledger=True also the
    build_info ledger after every step (values [T, 2, 8, P], kinds [T, 2, 8, P])."""
    T = actions.shape[0]
    NP = cfg.n_nodes * cfg.n_products
    H = cfg.heap_capacity
    obs = np.zeros((T + 1, cfg.n_obs))
    rew = np.zeros(T)
    stock = np.zeros((T + 1, NP))
    tk = np.zeros((T + 1, NP, H), dtype=np.int32)
    val = np.zeros((T + 1, NP, H))
    size = np.zeros((T + 1, NP), dtype=np.int32)
    thr = np.asarray(lt_thr if lt_thr is not None else [0], dtype=np.uint32)
    acts = np.ascontiguousarray(actions, dtype=np.float32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    args = [ctypes.byref(cfg), nodes, p(thr), ctypes.c_uint64(seed), ctypes.c_uint32(env_id),
            ctypes.c_uint32(episode), ctypes.c_int32(T), p(acts), p(obs), p(rew), p(stock), p(tk), p(val), p(size)]
    if ledger or staged:
        led_v = np.zeros((T, 2, 8, cfg.n_products))
        led_k = np.zeros((T, 2, 8, cfg.n_products), dtype=np.int32)
        if nodes_kernel:  # the node-parallel phases with ledgers kept by node, reduced in node order
            rc = lib.sch_episode_nodes_ledger(*args, p(led_v), p(led_k), ctypes.c_int32(int(nodes_serial)))
            return rc, obs, rew, stock, (tk, val, size), (led_v, led_k)
        fn = lib.sch_episode_staged if staged else lib.sch_episode_ledger
        rc = fn(*args, p(led_v), p(led_k))
        return rc, obs, rew, stock, (tk, val, size), (led_v, led_k)
    fn = lib.sch_episode_nodes_serial if nodes_serial else lib.sch_episode_nodes if nodes_kernel else lib.sch_episode_level if level else lib.sch_episode
    rc = fn(*args)
    return rc, obs, rew, stock, (tk, val, size)
