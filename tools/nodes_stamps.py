"""Where a node-parallel SupplyChain kernel wave spends its time (diagnostic build only).

    python tools/exp_build.py nstamps --reuse-objs -D SCG_NODES_STAMPS
    SCG_PKG_ROOT=exp/nstamps python tools/nodes_stamps.py [--envs 65536] [--steps 3]

Runs sc-2perstage-v0 steps with kernel="nodes"; after each, reads the shader-clock stamps
lane 0 of every wave wrote (scg_sc_nodes.hip NSTAMP: 0 start, 5 heaps staged, 6 past the
first barrier, 1 acted, 2 past the second, 3 heaps done, 7 past the third, 4 end) and prints per phase the median / p90 over waves, split by
wave index in the block (wave w runs node w), and the spread of wave starts and ends
(shader clocks, relative to the earliest start); then the clocks each wave spent in the
sections of its act and heaps phases (sections_by_wave_p50, from the SCG_ACCP section stamps). With a
persistent grid each wave's stamps are its last tile's: use --envs <= 64 x the resident
blocks (32,768 on MI355X) for one tile per block.
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dump", default="", help="also save every wave's stamps to DUMP_<step>.npz")
    ap.add_argument("--build-info", action="store_true",
                    help="the ledger instantiation (its reduce falls in the 'out' phase: stamps 7 -> 4)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import gym_supplychain_amd as gsa
    from gym_supplychain_amd import _native as nat
    fn = nat.lib.scg_nodes_debug_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    env = gsa.make_vec("sc-2perstage-v0", a.envs, seed=0, device=dev, obs_dtype=torch.float32, auto_reset=True,
                       kernel="nodes", build_info=a.build_info)
    W = env._cfg.group
    waves = (a.envs + 63) // 64 * W
    env.reset()
    gen = torch.Generator(device=dev).manual_seed(0)
    for _ in range(10):
        env.step(torch.rand((a.envs, env.n_actions), generator=gen, device=dev) * 2 - 1)
    buf = np.zeros((min(waves, 1 << 14), 28), dtype=np.uint64)
    for s in range(a.steps):
        act = torch.rand((a.envs, env.n_actions), generator=gen, device=dev) * 2 - 1
        torch.cuda.synchronize()
        env.step(act)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data, buf.shape[0]) == 0
        st = buf.astype(np.int64)
        # a persistent grid writes one record per (resident block, wave): the rest stay zero
        st = st[st[:, 4] != 0]
        t0 = st[:, 0].min()
        rel = st[:, :8] - t0
        out = {"step": s, "build_info": a.build_info, "waves": int(len(st)), "span": int(rel[:, 4].max()),
               "start_p50_p90_max": [int(np.percentile(rel[:, 0], q)) for q in (50, 90, 100)],
               "end_p10_p50_max": [int(np.percentile(rel[:, 4], q)) for q in (10, 50, 100)]}
        names = ["stage", "barrier0", "act", "barrier1", "heaps", "reward+barrier2", "out", "whole"]
        d = np.stack([rel[:, 5] - rel[:, 0], rel[:, 6] - rel[:, 5], rel[:, 1] - rel[:, 6], rel[:, 2] - rel[:, 1],
                      rel[:, 3] - rel[:, 2], rel[:, 7] - rel[:, 3], rel[:, 4] - rel[:, 7], rel[:, 4] - rel[:, 0]], 1)
        out["phase_p50_p90"] = {n: [int(np.percentile(d[:, k], 50)), int(np.percentile(d[:, k], 90))]
                                for k, n in enumerate(names)}
        wi = np.arange(len(st)) % W
        out["by_wave_p50"] = bw = {n: [int(np.median(d[wi == w, k])) for w in range(W)] for k, n in enumerate(names)}
        # The step's dependency graph against its barrier schedule (per-wave p50, wave w = node
        # w): the barriers make a tile cost the sum over phases of the slowest wave; without
        # them, a node's heaps would wait only for its own act and its sources' acts (the
        # inbox), and a node's act for the action tile and every wave's flags (barrier 0 stays).
        if W == 8 and a.envs >= 64:
            src = {2: (0, 1), 3: (0, 1), 4: (2, 3), 5: (2, 3), 6: (4, 5), 7: (4, 5)}  # sc-2perstage
            S, A, Hh, O = bw["stage"], bw["act"], bw["heaps"], bw["out"]
            sched = max(S) + max(A) + max(Hh) + max(O)
            act_end = [max(S) + A[i] for i in range(W)]
            heaps_end = [max([act_end[i]] + [act_end[j] for j in src.get(i, ())]) + Hh[i] for i in range(W)]
            out["critical_path_clocks"] = {"barrier_schedule": int(sched),
                                           "dependency_graph_keeping_barrier0": int(max(heaps_end) + max(O)),
                                           "mean_wave_work": int(np.mean(S) + np.mean(A) + np.mean(Hh) + np.mean(O))}
        # real-time clock (100 MHz, one clock for the whole chip): the launch's timeline in us
        rt = (st[:, 8:10] - st[:, 8].min()) / 100.0
        blk = np.arange(len(st)) // W
        bs, be = np.array([rt[blk == b, 0].min() for b in range(blk.max() + 1)]), \
            np.array([rt[blk == b, 1].max() for b in range(blk.max() + 1)])
        out["timeline_us"] = {"span": float(rt[:, 1].max()),
                              "block_start_pct": [float(np.percentile(bs, q)) for q in (0, 25, 50, 75, 100)],
                              "block_end_pct": [float(np.percentile(be, q)) for q in (0, 25, 50, 75, 100)],
                              "block_dur_p50": float(np.median(be - bs)),
                              "clock_mhz": float(np.median(d[:, 7] / np.maximum(rt[:, 1] - rt[:, 0], 1e-3)))}
        # section stamps (slot 12 + k = the clock at the end of section k, this launch's only
        # when inside its phase): durations from the previous stamp of the same phase
        secs = {"act": (6, [(7, "recv_clear"), (8, "stockpen_supply"), (9, "ship_split"), (10, "ship_dests"),
                            (11, "ship_rest_or_retail"), (12, "holding"), (13, "cost_obs")], 1),
                "heaps": (2, [(0, "inbox_push"), (1, "pops"), (2, "supply_push"), (3, "bins_copyback")], 3)}
        sec_out = {}
        for ph, (s0, lst, s1) in secs.items():
            prev = st[:, s0].copy()
            for k, nm in lst:
                x = st[:, 12 + k]
                ok = (x >= st[:, s0]) & (x <= st[:, s1])
                dur = np.where(ok, x - prev, 0)
                prev = np.where(ok, x, prev)
                sec_out[f"{ph}.{nm}"] = [int(np.median(dur[wi == w])) for w in range(W)]
            sec_out[f"{ph}.tail"] = [int(np.median((st[:, s1] - prev)[wi == w])) for w in range(W)]
        out["sections_by_wave_p50"] = sec_out
        if a.dump:
            np.savez(f"{a.dump}_{s}.npz", stamps=st, W=W)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
