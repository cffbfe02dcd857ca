"""Where a drop-in env's step time goes with the step servers (diagnostic).

    python tools/server_latency_probe.py [--weeks 3500] [--sc-steps 720]

Times, per call on one MI355X: the bare C call (BeerGameEnv: scg_bg_server_post + _wait;
SupplyChain2perStageEnv: scg_sc_server_post + _wait — the _scgpu_fast bindings, no Python work
around them) and the whole facade step() (action conversion, the call, the overflow check, the
NumPy outputs). One JSON line each: median / p10 / p90 microseconds.
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

    steps = int(sys.argv[sys.argv.index("--sc-steps") + 1]) if "--sc-steps" in sys.argv else 720
    env = gsa.make("sc-2perstage-v0", seed=0)
    T = env.total_time_steps
    call = env._server.step
    act = np.zeros(env.action_space.shape, dtype=np.float32)
    raw, whole = [], []
    for ep in range(1 + steps // T):
        env.reset()
        env._act_np[0, :] = act
        for t in range(T):
            t0 = pc()
            r = call()
            raw.append(pc() - t0)
            assert r in (0, 1), r
    for ep in range(1 + steps // T):
        env.reset()
        for t in range(T):
            t0 = pc()
            env.step(act)
            whole.append(pc() - t0)
    print(json.dumps({"measure": "scg_sc_server post + wait C call (sc-2perstage)", **stats(raw[T:])}))
    print(json.dumps({"measure": "SupplyChain2perStageEnv.step (facade)", **stats(whole[T:]),
                      "server_block_launches": env._server.launches}))
    env.close()


if __name__ == "__main__":
    main()
