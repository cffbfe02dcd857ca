"""Where the host time of one BeerGameVecEnv.step() goes (bench config, 65,536 envs).

    python tools/host_overhead.py [--iters 2000]

Prints one JSON line of per-call host microseconds (no synchronisation inside the loops,
so these are submission costs while the GPU drains behind them):
  py_noop            Python loop calling a no-op C function (binding floor)
  fast_invalid       _scgpu_fast.bg_step rejected at argument validation (no launch)
  torch_tiny_launch  a tiny torch elementwise op (HIP launch floor as torch pays it)
  step_loop          the bench loop: env.step(week[env.week]) (kernel launched)
  step_loop_wall_us  same, wall time per step including the drain at the end
and the kernel time per step from kernel-stamped events for comparison, plus torch's device
copy of the step kernel's byte count (17.05 MB: half read, half written) and of 4x that,
as the practical bandwidth ceiling at this working-set size (back-to-back launches, so the
figure includes launch gaps; an upper bound on per-launch time).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def per_call(fn, iters):
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--envs", type=int, default=65536)
    a = ap.parse_args()
    import ctypes

    import torch

    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd import _native as nat
    dev = torch.device("cuda", 0)
    N, L, T = a.envs, bench.LEVELS, bench.WEEKS
    env = BeerGameVecEnv(N, {}, demand="poisson", poisson_lambda=bench.LAMBDA, seed=bench.SEED, device=dev,
                         auto_reset=True, track_costs=True, track_history=True, track_returns=True)
    acts = torch.zeros((T, N, L), dtype=torch.int32, device=dev)
    week = list(acts.unbind(0))
    env.reset()
    out = {}
    noop = ctypes.CDLL(None).getpid
    out["py_noop"] = per_call(noop, a.iters)
    fast = nat.fast.bg_step
    out["fast_invalid"] = per_call(lambda: fast(0, 0, 0, 0, 0, 0, 0, 0), a.iters)
    x = torch.zeros(16, device=dev)
    torch.cuda.synchronize()
    out["torch_tiny_launch"] = per_call(lambda: x.add_(1), a.iters)
    torch.cuda.synchronize()
    for _ in range(70):
        env.step(week[env.week])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        env.step(week[env.week])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["step_loop"] = (t1 - t0) / a.iters * 1e6
    out["step_loop_wall_us"] = (t2 - t0) / a.iters * 1e6
    # the C entry point alone, arguments prepared (no Python wrapper): binding + library + HIP launch
    args = (env._cfg_addr, env._st_addr, week[0].data_ptr(), env._obs_ptr, env._rew_ptr, env._term_ptr, env._flags,
            nat.raw_stream(0))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        fast(*args)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    out["fast_direct"] = (t1 - t0) / a.iters * 1e6
    ev = [(nat.hip_event(), nat.hip_event()) for _ in range(200)]
    for e in ev:
        env.step(week[env.week], e)
    torch.cuda.synchronize()
    out["kernel_us"] = sum(nat.hip_event_elapsed_ms(s, e) for s, e in ev) / len(ev) * 1e3
    for s, e in ev:
        nat.hip_event_destroy(s)
        nat.hip_event_destroy(e)
    # practical ceiling at this size: torch's own copy of the same byte count (half read,
    # half written) and a 4x larger one, timed with events on the current stream
    for tag, nbytes in (("copy_same_bytes", 17054339), ("copy_4x_bytes", 4 * 17054339)):
        n = nbytes // 8
        src = torch.ones(n, dtype=torch.int32, device=dev)
        dst = torch.empty_like(src)
        for _ in range(20):
            dst.copy_(src)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(200):
            dst.copy_(src)
        s1.record()
        torch.cuda.synchronize()
        us = s0.elapsed_time(s1) / 200 * 1e3
        out[tag] = {"bytes": 2 * n * 4, "us": us, "GBps": 2 * n * 4 / us / 1e3}
    out["n_envs"] = N
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
