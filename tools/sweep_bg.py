"""BeerGame N-sweep: step kernel and rollout kernel from 65,536 envs past the Infinity Cache.

    python tools/sweep_bg.py [--max-log2 24] [--steps 70]

For each N prints one JSON line: Python-loop env-steps/s, step-kernel time (kernel-
stamped hipExtLaunchKernel events), algorithmic GB/s of the step kernel (bench.py's byte
model), and the K=35-week rollout kernel's env-steps/s and GB/s (36 B in/out per env-week
plus the ring row and the per-launch state). Same workload as bench.py (Poisson(8)
demand, uniform [0,8] actions, ledgers + history + returns, auto-reset).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)

import bench  # noqa: E402  (byte model)


def one(N, steps):
    import ctypes

    import torch

    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd import _native as nat
    dev = torch.device("cuda", 0)
    L, T = bench.LEVELS, bench.WEEKS
    env = BeerGameVecEnv(N, {}, demand="poisson", poisson_lambda=bench.LAMBDA, seed=bench.SEED, device=dev,
                         auto_reset=True, track_costs=True, track_history=True, track_returns=True)
    stream = torch.cuda.current_stream(dev)
    acts = torch.empty((T, N, L), dtype=torch.int32, device=dev)
    nat.check(nat.lib.scg_uniform_ints(bench.SEED, 0, N, T, L, 0, 0, 8, acts.data_ptr(),
                                       ctypes.c_void_p(stream.cuda_stream)))
    week = list(acts.unbind(0))
    env.reset()
    for _ in range(T):
        env.step(week[env.week])
    plan = list(env._plan)
    w0 = env.week
    nbytes = sum(N * bench.step_bytes_per_env(plan[(w0 + i) % T + 1], (w0 + i) % T + 1, T, L, 2, True, True, True,
                                              True) for i in range(steps))
    ev = [(nat.hip_event(), nat.hip_event()) for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        env.step(week[env.week], ev[i])
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern = sum(nat.hip_event_elapsed_ms(s, e) for s, e in ev) / 1e3
    for s, e in ev:
        nat.hip_event_destroy(s)
        nat.hip_event_destroy(e)
    # rollout: one full episode (35 weeks) per launch from week 0
    env.reset()
    obs = torch.empty((T, N, L), dtype=torch.int32, device=dev)
    rew = torch.empty((T, N), dtype=torch.int32, device=dev)
    env.rollout(acts, obs, rew)  # warm
    reps = max(1, steps // T)
    s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_ev.record(stream)
    for _ in range(reps):
        env.rollout(acts, obs, rew)
    e_ev.record(stream)
    torch.cuda.synchronize()
    roll_s = s_ev.elapsed_time(e_ev) / 1e3 / reps
    roll_bytes = N * (T * (16 + 16 + 4 + 16 + 16 + 16) + 2 * (3 * 16 + 2 * 16 + 8))  # act,obs,rew,ring r/w,hist + state
    out = {"n_envs": N, "python_loop_env_steps_per_s": N * steps / wall, "ms_per_step": wall * 1e3 / steps,
           "step_kernel_us": kern / steps * 1e6, "step_kernel_gbs": nbytes / kern / 1e9,
           "step_bytes_per_launch": nbytes / steps,
           "rollout_env_steps_per_s": N * T / roll_s, "rollout_kernel_us_per_episode": roll_s * 1e6,
           "rollout_gbs": roll_bytes / roll_s / 1e9}
    del env, acts, obs, rew
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-log2", type=int, default=16)
    ap.add_argument("--max-log2", type=int, default=24)
    ap.add_argument("--steps", type=int, default=70)
    a = ap.parse_args()
    for k in range(a.min_log2, a.max_log2 + 1):
        print(json.dumps(one(2 ** k, a.steps)), flush=True)


if __name__ == "__main__":
    main()
