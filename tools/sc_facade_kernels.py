"""SupplyChain2perStageEnv.step latency per kernel choice (diagnostic): the facade built with
kernel lane / nodes / staged, 3 episodes of 360 steps each, median of the last two; the last
episode's reward and observation sums must agree across kernels."""
import json, os, sys, time
sys.path.insert(0, "gym-supplychain_amd")
import numpy as np
import gym_supplychain_amd as gsa
from gym_supplychain_amd.envs import supplychain_env as se
orig = se.SupplyChainVecEnv.__init__
for k in ["lane", "nodes", "staged"]:
    def patched(self, *a, _k=k, **kw):
        kw["kernel"] = _k
        return orig(self, *a, **kw)
    se.SupplyChainVecEnv.__init__ = patched
    try:
        env = gsa.make("sc-2perstage-v0", seed=0)
    except Exception as e:
        print(k, "failed", e); continue
    rng = np.random.RandomState(0)
    acts = [rng.uniform(-1, 1, env.action_space.shape).astype(np.float32) for _ in range(720)]
    ts = []
    obs_all = []
    for ep in range(3):
        env.reset()
        for w in range(360):
            t0 = time.perf_counter(); o, r, d, _ = env.step(acts[(ep * 360 + w) % 720]); ts.append(time.perf_counter() - t0)
            if ep == 2: obs_all.append((o.copy(), r))
    ts = np.array(ts[360:]) * 1e6
    print(json.dumps({"kernel": env._vec.kernel, "median_us": float(np.median(ts)), "p90_us": float(np.percentile(ts, 90)),
                      "checksum": float(sum(float(x[1]) for x in obs_all)), "obs_sum": float(sum(x[0].sum() for x in obs_all))}))
