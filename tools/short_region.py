"""Wall time of the driver's short timed region (`bench.py --steps 20 --warmup 5`), repeated.

    [SCG_PKG_ROOT=exp/NAME] python tools/short_region.py [--label L] [--spin] [--steps 20] [--reps 30]

Per rep: barrier-free version of bench.region — synchronize, K steps, synchronize — after
one warm-up episode; prints one JSON line with the median / min wall per step, the median
GPU span per step (first launch's begin to last launch's end) and the host submit cost of
the C entry point alone. --spin sets hipDeviceScheduleSpin before the GPU is first touched
(the host thread spins instead of sleeping in synchronize).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="tree")
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch
    if a.spin:
        lib = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        hip = ctypes.CDLL(lib if os.path.exists(lib) else "libamdhip64.so.7")
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
        assert rc == 0, rc

    import bench
    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd import _native as nat
    dev = torch.device("cuda", 0)
    N, K, T = 65536, a.steps, bench.WEEKS
    env = BeerGameVecEnv(N, {}, demand="poisson", poisson_lambda=bench.LAMBDA, seed=bench.SEED, device=dev,
                         auto_reset=True, track_costs=True, track_history=True, track_returns=True)
    acts = torch.randint(0, 9, (T, N, 4), dtype=torch.int32, device=dev)
    loop = bench.StepLoop(env, list(acts.unbind(0)))
    env.reset()
    loop.run(T)
    walls, spans = [], []
    e0, e1 = nat.hip_event(), nat.hip_event()
    for _ in range(a.reps):
        wall, span = bench.region(loop, K, 1, None, torch.cuda.synchronize, (e0, e1, nat.hip_event_elapsed_ms))
        walls.append(wall * 1e6 / K)
        spans.append(span * 1e3 / K)
    args = (env._cfg_addr, env._st_addr, acts[0].data_ptr(), env._obs_ptr, env._rew_ptr, env._term_ptr, env._flags,
            nat.raw_stream(0))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2000):
        nat.fast.bg_step(*args)
    c_us = (time.perf_counter() - t0) / 2000 * 1e6
    torch.cuda.synchronize()
    print(json.dumps(dict(label=a.label, spin=a.spin, steps=K, wall_us_median=statistics.median(walls),
                          wall_us_min=min(walls), span_us_median=statistics.median(spans),
                          env_steps_per_s_median=N / (statistics.median(walls) / 1e6), c_entry_us=c_us)), flush=True)


if __name__ == "__main__":
    main()
