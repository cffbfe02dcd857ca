"""Where a SupplyChain LDS lane-kernel wave spends its time (diagnostic build only).

    python tools/exp_build.py stamps -D SCG_SC_STAMPS
    SCG_PKG_ROOT=exp/stamps python tools/sc_stamps.py [--envs 65536] [--steps 5]

Runs sc-2perstage-v0 steps; after each, reads the shader-clock stamps lane 0 of every wave
wrote at phase boundaries (scg_supplychain.hip SCG_STAMP: 0 start, 1 heaps staged,
2+i after node i's act, 23 return stored, 24 observation written, 25 heaps stored back)
and prints, per phase, the median / p90 cycles over waves, plus the spread of wave start
and end times across the launch (all in shader clocks, relative to the earliest start).
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--scenario", default="sc-2perstage-v0")
    ap.add_argument("--kernel", default="lane", help="lane (phase stamps) or staged (phase accumulators)")
    ap.add_argument("--nodes-per-echelon", default=None, help="e.g. 8,8,8,16 for sc-Nperstage-multiproduct-v0")
    a = ap.parse_args()
    import numpy as np
    import torch
    import gym_supplychain_amd as gsa
    from gym_supplychain_amd import _native as nat
    fn = nat.lib.scg_sc_debug_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    kw = {}
    if a.nodes_per_echelon:
        kw["nodes_per_echelon"] = [int(x) for x in a.nodes_per_echelon.split(",")]
    env = gsa.make_vec(a.scenario, a.envs, seed=0, device=dev, obs_dtype=torch.float32, auto_reset=True,
                       kernel=a.kernel, **kw)
    sym = env.kernel_symbol
    epb = int(sym.rsplit(",", 1)[1].rstrip(">")) if "lds" in sym else 64
    waves = (a.envs + epb - 1) // epb
    nn = len(env.spec.nodes)
    env.reset()
    gen = torch.Generator(device=dev).manual_seed(0)
    for _ in range(10):
        env.step(torch.rand((a.envs, env.n_actions), generator=gen, device=dev) * 2 - 1)
    buf = np.zeros((min(waves, 1 << 16), 32), dtype=np.uint64)
    for s in range(a.steps):
        act = torch.rand((a.envs, env.n_actions), generator=gen, device=dev) * 2 - 1
        torch.cuda.synchronize()
        env.step(act)
        torch.cuda.synchronize()
        rc = fn(buf.ctypes.data, buf.shape[0])
        assert rc == 0, rc
        st = buf.astype(np.int64)
        if a.kernel == "staged":  # accumulators in slots 16..23 (scg_supplychain_staged.h SCG_ACC)
            names = ["heap_copy_in", "drain_pushes", "receive_pops", "supply_push", "bins_copyback", "act_tail",
                     "stock_obs", "other", "act_pre_ship", "act_loads_split", "act_dest_loop", "act_post_ship",
                     "x12", "x13", "x14", "x15"]
            tot = st[:, 16:32].sum(axis=1)
            print(json.dumps({"step": s, "kernel": sym, "waves": int(buf.shape[0]),
                              "acc_total_med": int(np.median(tot)),
                              "share": {n: round(float(np.median(st[:, 16 + k] / tot)), 4) for k, n in enumerate(names)},
                              "cycles_med": {n: int(np.median(st[:, 16 + k])) for k, n in enumerate(names)}}),
                  flush=True)
            continue
        t0 = st[:, 0].min()
        marks = [0, 1] + [2 + min(i, 20) for i in range(nn)] + [23, 24, 25]
        names = ["stage_in"] + [f"node{i}" for i in range(nn)] + ["return", "observe", "stage_out"]
        out = {"step": s, "kernel": sym, "waves": int(buf.shape[0]),
               "start_spread": [int(np.percentile(st[:, 0] - t0, q)) for q in (0, 50, 90, 100)],
               "end": [int(np.percentile(st[:, 25] - t0, q)) for q in (0, 50, 90, 100)],
               "wave_total_med": int(np.median(st[:, 25] - st[:, 0]))}
        ph = {}
        for k in range(1, len(marks)):
            d = st[:, marks[k]] - st[:, marks[k - 1]]
            ph[names[k - 1]] = [int(np.median(d)), int(np.percentile(d, 90))]
        out["phases_med_p90"] = ph
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
