"""Host cost of the end-of-episode return all-gather (EpisodeReturnGather.on_episode_end) in
the bench's shape (65,536 int64 returns per rank), with a BeerGame step launched between
calls as in the step loop.

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \\
        --master-port 29540 tools/gather_probe.py [--iters 300]

Prints one JSON line per rank: us per on_episode_end call (median, mean), us per step
launch alone for comparison, and the same with a step between gathers.
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--envs", type=int, default=65536)
    a = ap.parse_args()
    import gc

    import torch
    import torch.distributed as dist

    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd.distributed import EpisodeReturnGather, shard_offset
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    rank, world = dist.get_rank(), dist.get_world_size()
    N, L, T = a.envs, bench.LEVELS, bench.WEEKS
    env = BeerGameVecEnv(N, {}, demand="poisson", poisson_lambda=bench.LAMBDA, seed=bench.SEED, device=dev,
                         env_offset=shard_offset(N, rank), auto_reset=True, track_costs=True, track_history=True,
                         track_returns=True)
    acts = torch.zeros((T, N, L), dtype=torch.int32, device=dev)
    week = list(acts.unbind(0))
    env.reset()
    gather = EpisodeReturnGather(N, dev, collective=True)
    ret = env._final_ret if getattr(env, "_final_ret", None) is not None else torch.zeros(N, dtype=torch.int64,
                                                                                          device=dev)
    for _ in range(50):
        env.step(week[env.week])
        gather.on_episode_end(ret)
    gather.result()
    torch.cuda.synchronize()
    gc.disable()
    g, s = [], []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        env.step(week[env.week])
        t1 = time.perf_counter()
        gather.on_episode_end(ret)
        t2 = time.perf_counter()
        s.append((t1 - t0) * 1e6)
        g.append((t2 - t1) * 1e6)
        if len(g) % 20 == 0:
            torch.cuda.synchronize()
    gather.result()
    torch.cuda.synchronize()
    gc.enable()
    print(json.dumps({"rank": rank, "world": world, "gather_us_median": statistics.median(g),
                      "gather_us_mean": statistics.fmean(g), "step_us_median": statistics.median(s),
                      "impl": "rccl" if gather._rccl is not None else "torch",
                      "out_ok": bool((gather.result()[:N] == ret).all())}), flush=True)
    r = gather._rccl
    if r is not None:  # the RCCL path's parts, each timed alone
        import ctypes

        from gym_supplychain_amd import _native as nat
        from gym_supplychain_amd.distributed import _async_copy
        s = nat.raw_stream(local)
        parts = {}

        def timed(name, fn):
            torch.cuda.synchronize()
            t = []
            for _ in range(a.iters):
                t0 = time.perf_counter()
                fn()
                t.append((time.perf_counter() - t0) * 1e6)
                if len(t) % 20 == 0:
                    torch.cuda.synchronize()
            parts[name] = statistics.median(t)
        timed("copy", lambda: _async_copy(gather._stage, ret))
        timed("copy_direct", lambda: r.hip.hipMemcpyAsync(gather._stage.data_ptr(), ret.data_ptr(), N * 8, 3, s))
        timed("record", lambda: r.hip.hipEventRecord(r.ready, s))
        timed("wait", lambda: r.hip.hipStreamWaitEvent(r.gstream, r.ready, 0))
        timed("record_wait", lambda: (r.hip.hipEventRecord(r.ready, ctypes.c_void_p(s)),
                                      r.hip.hipStreamWaitEvent(r.gstream, r.ready, 0)))
        timed("allgather", lambda: r.lib.ncclAllGather(gather._stage.data_ptr(), gather._out.data_ptr(),
                                                       gather._stage.numel(), r.NCCL_INT64, r.comm, r.gstream))
        timed("allgather_same_stream", lambda: r.lib.ncclAllGather(gather._stage.data_ptr(), gather._out.data_ptr(),
                                                                   gather._stage.numel(), r.NCCL_INT64, r.comm,
                                                                   ctypes.c_void_p(s)))
        print(json.dumps({"rccl_parts_us_median": parts}), flush=True)
    gather.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
