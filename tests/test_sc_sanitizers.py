"""Host sanitizer build: the SupplyChain kernel bodies — lane, level, staged
(with build_info ledgers), the node-parallel phases with the nodes in REVERSE order and the
node-parallel serial walk, plus the lane body with ledgers — compiled for the host with
AddressSanitizer and UndefinedBehaviorSanitizer (tests/native/sc_host_asan_main.cpp) and run
over every golden SupplyChain case. The run must be clean (any report aborts the process
with a non-zero status) and every result must still equal the reference's vectors.

The sanitized program runs as a child process, so nothing is preloaded into pytest's own.
GPU sanitizers are not available on the pool; this is the host half.
"""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from conftest import PKG_ROOT, REPO
from golden_io import load_sc, sc_cases

SRC = os.path.join(REPO, "tests", "native", "sc_host_asan_main.cpp")
HARNESS = os.path.join(REPO, "tests", "native", "sc_host_harness.cpp")
EXE = os.path.join(REPO, "tests", "native", "_build", "sc_host_asan")
CSRC = os.path.join(PKG_ROOT, "csrc")
MODES = {"lane": 0, "level": 1, "staged": 2, "nodes_reverse": 3, "nodes_serial": 4, "lane_ledger": 5}
ENVS_PER_CASE = 2


def build():
    deps = [SRC, HARNESS] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
        [os.path.join(REPO, "include", "scgpu.h")]
    if os.path.exists(EXE) and all(os.path.getmtime(EXE) >= os.path.getmtime(d) for d in deps):
        return EXE
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    # -fsanitize only for the host compilation (the device side has no sanitizer here)
    tmp = f"{EXE}.{os.getpid()}.tmp"  # concurrent test workers: build aside, rename into place
    subprocess.run([hipcc, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-ffp-contract=off",
                    "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                    "-Xarch_host", "-fno-sanitize-recover=all", "-Wno-pass-failed", "--offload-arch=gfx950",
                    "-I", os.path.join(REPO, "include"), "-I", CSRC, "-I", os.path.dirname(SRC),
                    "-o", tmp, SRC], check=True)
    os.replace(tmp, EXE)
    return EXE


def _job(mode, c, nodes, thr, seed, env_id, episode, actions):
    import ctypes
    steps, A = actions.shape
    NP, H, P = c.n_nodes * c.n_products, c.heap_capacity, c.n_products
    thr = np.asarray(thr if thr is not None else [], dtype=np.uint32)
    keep = getattr(c, "_keep", [])
    dthr = next((a for a in keep if a.dtype == np.uint32), np.zeros(0, np.uint32)) if c.demand_thr else np.zeros(0, np.uint32)
    dbase = next((a for a in keep if a.dtype == np.float64), np.zeros(0)) if c.demand_base else np.zeros(0)
    head = struct.pack("<14i", 0x53434A42, mode, ctypes.sizeof(c), ctypes.sizeof(nodes[0]), c.n_nodes, len(thr),
                       len(dthr), len(dbase), steps, A, c.n_obs, NP, H, P)
    head += struct.pack("<QII", seed, env_id, episode)
    return (head + bytes(c) + bytes(nodes) + thr.tobytes() + dthr.astype(np.uint32).tobytes() +
            dbase.astype(np.float64).tobytes() + np.ascontiguousarray(actions, dtype=np.float32).tobytes())


def _read_result(buf, off, steps, O, NP, H, P):
    def take(dtype, count):
        nonlocal off
        a = np.frombuffer(buf, dtype=dtype, count=count, offset=off)
        off += a.nbytes
        return a
    rc, fallbacks = take(np.int32, 2)
    r = dict(rc=int(rc), fallbacks=int(fallbacks), obs=take(np.float64, (steps + 1) * O).reshape(steps + 1, O),
             rew=take(np.float64, steps), stock=take(np.float64, (steps + 1) * NP).reshape(steps + 1, NP))
    r["tk"] = take(np.int32, (steps + 1) * NP * H).reshape(steps + 1, NP, H)
    r["val"] = take(np.float64, (steps + 1) * NP * H).reshape(steps + 1, NP, H)
    r["size"] = take(np.int32, (steps + 1) * NP).reshape(steps + 1, NP)
    r["led_v"] = take(np.float64, steps * 16 * P).reshape(steps, 2, 8, P)
    r["led_k"] = take(np.int32, steps * 16 * P).reshape(steps, 2, 8, P)
    return r, off


@pytest.mark.parametrize("name", sc_cases())
def test_sanitized_kernel_bodies_match_reference(name, tmp_path):
    from gym_supplychain_amd import _native as nat
    from test_sc_host import _setup
    exe = build()
    g = load_sc(name)
    seed = g["meta"]["seed"]
    N = min(ENVS_PER_CASE, g["obs"].shape[1])
    kernels = {0: nat.SC_KERNEL_LANE, 1: nat.SC_KERNEL_LEVEL, 2: nat.SC_KERNEL_STAGED, 3: nat.SC_KERNEL_STAGED,
               4: nat.SC_KERNEL_STAGED, 5: nat.SC_KERNEL_LANE}
    setups = {m: _setup(g, k) for m, k in kernels.items()}
    jobs, order = [], []
    for m, (spec, c, nodes, thr) in setups.items():
        for n in range(N):
            jobs.append(_job(m, c, nodes, thr, seed, n, 0, g["actions"][:, n]))
            order.append((m, n))
    jf, of = tmp_path / "jobs.bin", tmp_path / "out.bin"
    jf.write_bytes(b"".join(jobs))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    proc = subprocess.run([exe, str(jf), str(of)], capture_output=True, text=True, env=env, timeout=600)
    assert proc.returncode == 0, proc.stderr[-4000:]
    assert "runtime error" not in proc.stderr and "ERROR: AddressSanitizer" not in proc.stderr, proc.stderr[-4000:]
    buf, off = of.read_bytes(), 0
    for (m, n) in order:
        spec, c, _, _ = setups[m]
        steps = g["actions"].shape[0]
        NP, H, P = c.n_nodes * c.n_products, c.heap_capacity, c.n_products
        r, off = _read_result(buf, off, steps, c.n_obs, NP, H, P)
        assert r["rc"] == 0, (name, m, n)
        assert np.array_equal(r["obs"], g["obs"][:, n]), (name, m, n)
        assert np.array_equal(r["rew"], g["reward"][:, n]), (name, m, n)
        assert np.array_equal(r["stock"].reshape(steps + 1, -1, P), g["stock"][:, n]), (name, m, n)
        gt = g["heap_t"][:, n].reshape(steps + 1, -1, g["heap_t"].shape[-1])
        gv = g["heap_v"][:, n].reshape(gt.shape)
        for s_ in range(steps + 1):
            for hp in range(gt.shape[1]):
                k = int(r["size"][s_, hp])
                assert (r["tk"][s_, hp, :k] >> 3).tolist() == gt[s_, hp, :k].tolist(), (name, m, n, s_)
                assert r["val"][s_, hp, :k].tolist() == gv[s_, hp, :k].tolist(), (name, m, n, s_)
        if m >= 2:
            assert np.array_equal(r["led_v"][:, 0], g["led_cost"][:, n]), (name, m, n)
            assert np.array_equal(r["led_v"][:, 1], g["led_units"][:, n]), (name, m, n)
            assert np.array_equal(r["led_k"][:, 0], g["led_cost_k"][:, n]), (name, m, n)
            assert np.array_equal(r["led_k"][:, 1], g["led_units_k"][:, n]), (name, m, n)
    assert off == len(buf)
