"""Where the BeerGame step kernel's time goes at small batch sizes: its duration against
the batch size, isolated (one launch at a time, GPU idle in between) and back-to-back
(launches queued behind each other, as in bench.py), next to torch's device copy of the
same byte count and a 1-element fill (the launch floor).

    python tools/floor_probe.py [--min-log2 10] [--max-log2 18]

One JSON line per N.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-log2", type=int, default=10)
    ap.add_argument("--max-log2", type=int, default=18)
    ap.add_argument("--launches", type=int, default=700)
    a = ap.parse_args()
    import torch

    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd import _native as nat
    dev = torch.device("cuda", 0)
    L, T = bench.LEVELS, bench.WEEKS

    def timed(fn, k):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(20):
            fn()
        s.record()
        for _ in range(k):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / k * 1e3

    x = torch.zeros(1, device=dev)
    fill_us = timed(lambda: x.fill_(1.0), 500)
    for k in range(a.min_log2, a.max_log2 + 1):
        N = 2 ** k
        env = BeerGameVecEnv(N, {}, demand="poisson", poisson_lambda=bench.LAMBDA, seed=bench.SEED, device=dev,
                             auto_reset=True, track_costs=True, track_history=True, track_returns=True)
        acts = torch.randint(0, 9, (T, N, L), dtype=torch.int32, device=dev)
        week = list(acts.unbind(0))
        env.reset()
        for _ in range(70):
            env.step(week[env.week])
        # isolated: wait for each launch before the next
        ev = [(nat.hip_event(), nat.hip_event()) for _ in range(a.launches)]
        for e in ev[:200]:
            env.step(week[env.week], e)
            torch.cuda.synchronize()
        iso = sum(nat.hip_event_elapsed_ms(s, e) for s, e in ev[:200]) / 200 * 1e3
        # back-to-back: every 7th launch stamped, the rest queued behind it
        torch.cuda.synchronize()
        used = 0
        for i in range(a.launches):
            if i % 7 == 0:
                env.step(week[env.week], ev[used])
                used += 1
            else:
                env.step(week[env.week])
        torch.cuda.synchronize()
        b2b = sum(nat.hip_event_elapsed_ms(s, e) for s, e in ev[:used]) / used * 1e3
        wall = timed(lambda: env.step(week[env.week]), a.launches)
        for s, e in ev:
            nat.hip_event_destroy(s)
            nat.hip_event_destroy(e)
        nbytes = 17054339.657 * N / 65536
        n = int(nbytes // 8)
        src = torch.ones(n, dtype=torch.int32, device=dev)
        dst = torch.empty_like(src)
        copy_us = timed(lambda: dst.copy_(src), 300)
        print(json.dumps({"n_envs": N, "step_isolated_us": iso, "step_back_to_back_us": b2b,
                          "step_wall_us": wall, "copy_same_bytes_us": copy_us, "fill1_us": fill_us,
                          "bytes": nbytes}), flush=True)
        del env, acts, week, src, dst
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
