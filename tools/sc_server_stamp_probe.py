"""Where the SupplyChain step server's per-step time goes on the device (diagnostic; an
experiment build that stamps the block, tools/exp_build.py scstamp with the --replace edits
named in profiles/r06k_sc_server_stamps.log):

    SCG_PKG_ROOT=exp/scstamp python tools/sc_server_stamp_probe.py

The block accumulates, per request, the 100 MHz real-time clock from the request seen to the
tile's end (every wave past a barrier) and from there through the release fence, in the
mailbox's answer-line pad words; the host times the C call around them.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))


def main():
    import numpy as np
    import gym_supplychain_amd as gsa
    env = gsa.make("sc-2perstage-v0", seed=0)
    T = env.total_time_steps
    call = env._server.step
    box = env._server.box
    act = np.zeros(env.action_space.shape, dtype=np.float32)
    env.reset()
    env._act_np[0, :] = act
    for t in range(T):
        call()
    for i in range(6):
        box.pad2[i] = 0
    raw = []
    pc = time.perf_counter
    for ep in range(2):
        env.reset()
        env._act_np[0, :] = act
        for t in range(T):
            t0 = pc()
            call()
            raw.append(pc() - t0)
    n = max(int(box.pad2[2]), 1)
    print(json.dumps({"requests": n, "c_call_median_us": float(np.median(raw) * 1e6),
                      "device_seen_to_tile_end_us": box.pad2[0] / n * 0.01,
                      "device_release_fence_us": box.pad2[1] / n * 0.01,
                      "of_which_workgroup_wait_us": box.pad2[3] / n * 0.01,
                      "agent_l2_writeback_us": box.pad2[4] / n * 0.01,
                      "system_writeback_us": box.pad2[5] / n * 0.01}))
    env.close()


if __name__ == "__main__":
    main()
