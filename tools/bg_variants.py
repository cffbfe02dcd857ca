"""Step-kernel time of BeerGame variants at the bench size, to see what the kernel's time
goes to: demand source (fixed list / Poisson via Philox + threshold walk / uniform via
Philox), optional outputs (ledgers, history, returns).

    python tools/bg_variants.py [--envs 65536] [--launches 700]

One JSON line per variant: mean kernel µs (kernel-stamped events on every launch; this
tool does not time the Python loop) and the algorithmic bytes per launch of bench.py's
byte model where it applies.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)

import bench  # noqa: E402

VARIANTS = [
    ("bench: poisson + ledgers + history + returns", dict(demand="poisson"), dict(track_history=True)),
    ("fixed demand, same outputs", dict(demand="fixed"), dict(track_history=True)),
    ("uniform demand (Philox, no table)", dict(demand=("uniform", 0, 16)), dict(track_history=True)),
    ("poisson, no history", dict(demand="poisson"), dict(track_history=False)),
    ("poisson, no ledgers/history/returns", dict(demand="poisson"),
     dict(track_history=False, track_costs=False, track_returns=False)),
    ("fixed, no ledgers/history/returns", dict(demand="fixed"),
     dict(track_history=False, track_costs=False, track_returns=False)),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=bench.N_ENVS)
    ap.add_argument("--launches", type=int, default=700)
    a = ap.parse_args()
    import torch

    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd import _native as nat
    dev = torch.device("cuda", 0)
    N, L, T = a.envs, bench.LEVELS, bench.WEEKS
    acts = torch.randint(0, 9, (T, N, L), dtype=torch.int32, device=dev)
    week = list(acts.unbind(0))
    for name, dkw, tkw in VARIANTS:
        kw = dict(track_costs=True, track_returns=True)
        kw.update(tkw)
        env = BeerGameVecEnv(N, {}, poisson_lambda=bench.LAMBDA, seed=bench.SEED, device=dev, auto_reset=True,
                             **dkw, **kw)
        env.reset()
        for _ in range(70):
            env.step(week[env.week])
        ev = [(nat.hip_event(), nat.hip_event()) for _ in range(a.launches)]
        for e in ev:
            env.step(week[env.week], e)
        torch.cuda.synchronize()
        us = sum(nat.hip_event_elapsed_ms(s, e) for s, e in ev) / len(ev) * 1e3
        for s, e in ev:
            nat.hip_event_destroy(s)
            nat.hip_event_destroy(e)
        print(json.dumps({"variant": name, "n_envs": N, "kernel_us": us}), flush=True)
        del env
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
