"""Where a short timed region's time goes (the driver's `bench.py --steps 20 --warmup 5`).

    python tools/startup_probe.py [--steps 20] [--reps 5]

After a warm-up episode and a synchronize, K steps are launched back to back with EVERY
launch stamped by hipExtLaunchKernel (its own dispatch begin / end), then synchronised.
Per rep, one JSON line: the wall time of the region, the host time to submit all K steps,
the offsets (µs from the region's start on the host clock is not available, so from the
first kernel's begin) of every kernel's begin and end, the gaps between consecutive
kernels and their durations — i.e. whether the GPU idles waiting for the host early in the
region, and how long the first launch takes to start.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--envs", type=int, default=65536)
    a = ap.parse_args()
    import torch

    import bench
    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd import _native as nat
    dev = torch.device("cuda", 0)
    N, K = a.envs, a.steps
    env = BeerGameVecEnv(N, {}, demand="poisson", poisson_lambda=bench.LAMBDA, seed=bench.SEED, device=dev,
                         auto_reset=True, track_costs=True, track_history=True, track_returns=True)
    acts = torch.randint(0, 9, (bench.WEEKS, N, bench.LEVELS), dtype=torch.int32, device=dev)
    week = list(acts.unbind(0))
    env.reset()
    for _ in range(bench.WEEKS):
        env.step(week[env.week])
    anchor = nat.hip_event()
    for rep in range(a.reps):
        evs = [(nat.hip_event(), nat.hip_event()) for _ in range(K)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            env.step(week[env.week], evs[i])
        t_sub = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        begin = [0.0] + [nat.hip_event_elapsed_ms(evs[0][0], evs[i][0]) * 1e3 for i in range(1, K)]
        end = [nat.hip_event_elapsed_ms(evs[0][0], evs[i][1]) * 1e3 for i in range(K)]
        dur = [e - b for b, e in zip(begin, end)]
        gaps = [begin[i + 1] - end[i] for i in range(K - 1)]
        print(json.dumps(dict(rep=rep, steps=K, wall_us=wall * 1e6, submit_us=t_sub * 1e6,
                              gpu_span_us=end[-1], wall_minus_span_us=wall * 1e6 - end[-1],
                              kernel_us=[round(x, 2) for x in dur], gap_us=[round(x, 2) for x in gaps])), flush=True)
        for s, e in evs:
            nat.hip_event_destroy(s)
            nat.hip_event_destroy(e)
    nat.hip_event_destroy(anchor)


if __name__ == "__main__":
    main()
