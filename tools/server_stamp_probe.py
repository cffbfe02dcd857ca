"""Where the BeerGame step server's per-step time goes on the device (diagnostic; an
experiment build that stamps the wave, tools/exp_build.py srvstamp with the --replace edits
named in profiles/r06i_server_stamps.log):

    SCG_PKG_ROOT=exp/srvstamp python tools/server_stamp_probe.py

The wave accumulates, per request, the 100 MHz real-time clock from the request seen to the
week body's end and across the release fence, and the polls it made since the previous
request, in the mailbox's control-line pad words; the host times the C call around them.
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
    env = gsa.make("beergame-v0")
    T = env.max_weeks
    call = env._server.step
    box = env._server.server.box
    pc = time.perf_counter
    for ep in range(3):  # warm-up
        env.reset()
        for w in range(T):
            call()
    for i in range(4):
        box.pad[i] = 0
    raw = []
    for ep in range(100):
        env.reset()
        env._act_np[:] = 1
        for w in range(T):
            t0 = pc()
            call()
            raw.append(pc() - t0)
    n = max(int(box.pad[2]), 1)
    print(json.dumps({"requests": n, "c_call_median_us": float(np.median(raw) * 1e6),
                      "device_seen_to_body_end_us": box.pad[0] / n * 0.01,
                      "device_release_fence_us": box.pad[1] / n * 0.01,
                      "polls_per_request": box.pad[3] / n}))
    env.close()


if __name__ == "__main__":
    main()
