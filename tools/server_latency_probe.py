"""Where a drop-in BeerGameEnv.step's time goes with the step server (diagnostic).

    python tools/server_latency_probe.py [--weeks 3500]

Times, per call on one MI355X: the bare C call scg_bg_server_step (post the week, spin until
the resident wave answers; the _scgpu_fast binding, no Python work around it) and the whole
facade step() (action conversion, the call, the overflow check, the NumPy outputs). One JSON
line each: median / p10 / p90 microseconds.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gym-supplychain_amd"))


def stats(ts):
    import numpy as np
    a = np.asarray(ts) * 1e6
    return {"median_us": float(np.median(a)), "p10_us": float(np.percentile(a, 10)),
            "p90_us": float(np.percentile(a, 90)), "calls": int(a.size)}


def main():
    import numpy as np
    import gym_supplychain_amd as gsa
    weeks = int(sys.argv[sys.argv.index("--weeks") + 1]) if "--weeks" in sys.argv else 3500
    env = gsa.make("beergame-v0")
    T = env.max_weeks
    pc = time.perf_counter
    raw, whole = [], []
    call = env._server.step
    for ep in range(2 + weeks // T):
        env.reset()
        env._act_np[:] = 1
        for w in range(T):
            t0 = pc()
            r = call()
            raw.append(pc() - t0)
            assert r in (0, 1), r
    for ep in range(2 + weeks // T):
        env.reset()
        for w in range(T):
            t0 = pc()
            env.step([1, 2, 3, 4])
            whole.append(pc() - t0)
    print(json.dumps({"measure": "scg_bg_server_step C call", **stats(raw[2 * T:])}))
    print(json.dumps({"measure": "BeerGameEnv.step (facade)", **stats(whole[2 * T:]),
                      "server_wave_launches": int(env._server.sv.launches)}))
    env.close()


if __name__ == "__main__":
    main()
