"""A/B of BeerGame step kernels at the bench size on one box.

    SCG_PKG_ROOT=exp/NAME python tools/bg_ab.py --label NAME [--envs 65536]

For the package at SCG_PKG_ROOT (default: the working tree) and each state layout the
package offers (slab / separate buffers), one JSON line: the mean isolated kernel time
(every launch stamped by hipExtLaunchKernel with its own dispatch begin/end and run alone),
the back-to-back GPU timeline per launch (events around 3500 unstamped launches) and the
wall time per step of that loop.
"""
import argparse
import inspect
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="tree")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--launches", type=int, default=3500)
    ap.add_argument("--isolated", type=int, default=700)
    a = ap.parse_args()
    import torch

    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd import _native as nat
    dev = torch.device("cuda", 0)
    N, L, T = a.envs, 4, 35
    acts = torch.randint(0, 9, (T, N, L), dtype=torch.int32, device=dev)
    week = list(acts.unbind(0))
    layouts = [True, False] if "state_slab" in inspect.signature(BeerGameVecEnv.__init__).parameters else [None]
    for slab in layouts:
        kw = {} if slab is None else dict(state_slab=slab)
        env = BeerGameVecEnv(N, {}, demand="poisson", poisson_lambda=8.0, seed=0x5EED0000, device=dev,
                             auto_reset=True, track_costs=True, track_history=True, track_returns=True, **kw)
        env.reset()
        for _ in range(350):
            env.step(week[env.week])
        torch.cuda.synchronize()
        evs = [(nat.hip_event(), nat.hip_event()) for _ in range(a.isolated)]
        for e in evs:
            env.step(week[env.week], e)
            torch.cuda.synchronize()
        iso = sum(nat.hip_event_elapsed_ms(s, e) for s, e in evs) / len(evs) * 1e3
        for s, e in evs:
            nat.hip_event_destroy(s)
            nat.hip_event_destroy(e)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for _ in range(a.launches):
            env.step(week[env.week])
        e1.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.launches * 1e6
        print(json.dumps(dict(label=a.label, slab=slab, n_envs=N, isolated_us=iso,
                              timeline_us=e0.elapsed_time(e1) * 1e3 / a.launches, wall_us=wall)), flush=True)


if __name__ == "__main__":
    main()
