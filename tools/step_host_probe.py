"""Host time of each BeerGameVecEnv.step call in short bench regions (diagnostic).

    python tools/step_host_probe.py [--regions 50] [--k 20]

Builds the bench's env and resident week actions (bench.GpuPlatform), then times `regions`
regions of k step calls, each after a torch.cuda.synchronize() (the bench brackets a region
that way), call by call with perf_counter. Prints the median host time per call index inside
a region, the median of terminal-week calls (auto-reset week: the return snapshot happens
there) and of the others: where a K = 20 region's host enqueue goes.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    import bench
    regions = int(sys.argv[sys.argv.index("--regions") + 1]) if "--regions" in sys.argv else 50
    k = int(sys.argv[sys.argv.index("--k") + 1]) if "--k" in sys.argv else 20
    plat = bench.GpuPlatform()
    env = plat.make_env(65536, 0)
    acts = plat.week_actions(env, 65536)
    env.reset()
    T = len(acts)
    per_idx = [[] for _ in range(k)]
    term, other = [], []
    pc = time.perf_counter
    for r in range(regions + 3):
        torch.cuda.synchronize()
        for i in range(k):
            w = env.week
            t0 = pc()
            info = env.step(acts[w])[3]
            dt = pc() - t0
            if r >= 3:
                per_idx[i].append(dt)
                (term if info else other).append(dt)
    torch.cuda.synchronize()
    med = lambda x: float(np.median(np.asarray(x) * 1e6)) if x else None
    print(json.dumps({"k": k, "regions": regions, "median_us_by_index": [round(med(x), 2) for x in per_idx],
                      "terminal_median_us": med(term), "terminal_calls": len(term), "other_median_us": med(other),
                      "region_mean_us_per_step": float(np.mean([sum(x) for x in zip(*per_idx)]) / k * 1e6)}))


if __name__ == "__main__":
    main()
