"""Where the SupplyChain step server's tile spends its time, per wave and phase (diagnostic
build only):

    python tools/exp_build.py nstamps --reuse-objs -D SCG_NODES_STAMPS
    SCG_PKG_ROOT=exp/nstamps python tools/sc_server_phase_probe.py [--episodes 2]

Steps the drop-in sc-2perstage-v0 env through its step server (one resident block, a wave
per node) over whole episodes with uniform [-1, 1] actions (the reference's action range)
and with zero actions, then reads the block's per-wave phase sums (scg_sc_server_debug_phases,
scg_sc_nodes.hip: request seen -> tile start, stage, barrier 0, act, barrier 1, heaps, barrier
2 (wave 0's reward inside), out, closing barrier) without a device synchronisation, and
prints the mean shader clocks per served step for every wave, beside the C call's median.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))

PHASES = ["seen_to_tile", "stage", "barrier0", "act", "barrier1", "heaps", "barrier2_reward", "out", "close_barrier"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    import gym_supplychain_amd as gsa
    from gym_supplychain_amd import _native as nat
    fn = nat.lib.scg_sc_server_debug_phases
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros((8, 10), dtype=np.uint64)
    env = gsa.make("sc-2perstage-v0", seed=0)
    T = env.total_time_steps
    call = env._server.step
    rng = np.random.default_rng(0)
    pc = time.perf_counter
    for mode in ("uniform", "zeros"):
        env.reset()  # warm-up episode (launches the block, settles the caches)
        for t in range(T):
            env._act_np[0, :] = rng.uniform(-1, 1, env._act_np.shape[1]) if mode == "uniform" else 0.0
            r = call()
            assert r in (0, 1), r
        nat.check(fn(buf.ctypes.data, 1))
        raw = []
        for ep in range(a.episodes):
            env.reset()
            for t in range(T):
                env._act_np[0, :] = rng.uniform(-1, 1, env._act_np.shape[1]) if mode == "uniform" else 0.0
                t0 = pc()
                r = call()
                raw.append(pc() - t0)
                assert r in (0, 1), r
        nat.check(fn(buf.ctypes.data, 1))
        st = buf.astype(np.float64)
        n = st[:, 9].max()
        waves = {f"wave{w}": {p: round(st[w, k] / max(st[w, 9], 1), 0) for k, p in enumerate(PHASES)}
                 for w in range(8) if st[w, 9] > 0}
        tile = {w: sum(v.values()) for w, v in waves.items()}
        print(json.dumps({"actions": mode, "steps_served": int(n), "c_call_median_us": float(np.median(raw) * 1e6),
                          "clocks_per_step_by_wave": waves, "seen_to_past_close_barrier_clocks": tile}))
    env.close()
    # where the block ran (the last tile's NSTAMP record of wave 0: HW_ID and XCC_ID registers)
    rec = np.zeros((8, 28), dtype=np.uint64)
    st = nat.lib.scg_nodes_debug_stamps
    st.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nat.check(st(rec.ctypes.data, 8))
    hw = int(rec[0, 10])
    print(json.dumps({"block_xcc_id": int(rec[0, 11]) & 0xF, "hw_id": hex(hw), "cu_id": (hw >> 8) & 0xF,
                      "sh_id": (hw >> 12) & 1, "se_id": (hw >> 13) & 0x7}))


if __name__ == "__main__":
    main()
