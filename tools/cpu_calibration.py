"""Calibrate bench.py's cpu_baseline worker against the reference — build container only.

    python tools/cpu_calibration.py [--seconds 6.0] [--reps 7] [--cpu K]

BASELINE.md:62 asks that the restatement timed on the GPU box (oracle.beergame.
BeerGameOracle, the "reference NumPy step()") run within +-15 % of the reference's own
BeerGameEnv per core. This times both with bench.py's worker loop on one core — per episode:
construct the env with that episode's customer_demand, reset(), 35 step() calls on
pre-drawn actions — alternating them `--reps` times (pinned to one core), and prints one JSON
line with both median rates, their ratio and the median of the per-pair ratios (each pair
ran back to back, so host drift cancels in it). The reference is imported read-only from /root/reference with the
gym stand-in of oracle/refharness/; without it the script exits.
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)


def rate(make_env, demands, acts, seconds):
    steps, ep = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        k = ep % len(demands)
        env = make_env({"customer_demand": demands[k]})
        env.reset()
        for w in range(35):
            env.step(acts[k, w])
        steps += 35
        ep += 1
    return steps / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--cpu", type=int, default=None, help="core to pin to (default: the last one available)")
    a = ap.parse_args()
    cpus = sorted(os.sched_getaffinity(0))
    os.sched_setaffinity(0, {cpus[-1] if a.cpu is None else a.cpu})
    if not os.path.isdir(REFERENCE):
        print(f"{REFERENCE} absent")
        return
    sys.path.insert(0, REFERENCE)
    sys.path.insert(0, os.path.join(REPO, "oracle", "refharness"))
    import numpy as np

    import bench
    from gym_supplychain.envs.beergame_env import BeerGameEnv  # reference, read-only
    from oracle.beergame import BeerGameOracle
    demands, acts = bench.cpu_worker_inputs(0, 64)
    ref, port = [], []
    for _ in range(a.reps):
        ref.append(rate(BeerGameEnv, demands, acts, a.seconds))
        port.append(rate(BeerGameOracle, demands, acts, a.seconds))
    pairs = [p / r for p, r in zip(port, ref)]
    out = dict(reference_steps_per_s=statistics.median(ref), port_steps_per_s=statistics.median(port),
               ratio_port_over_reference=statistics.median(port) / statistics.median(ref),
               median_pair_ratio=statistics.median(pairs), pair_ratios=pairs,
               within_15pct=all(0.85 <= x <= 1.15 for x in (statistics.median(pairs),)),
               reference_runs=ref, port_runs=port, cores=1, seconds_per_run=a.seconds,
               numpy=np.__version__, python=sys.version.split()[0])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
