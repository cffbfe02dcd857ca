"""Per-call latency of the drop-in single envs (gym.make("beergame-v0") / "sc-2perstage-v0"
users get these in place of the reference's classes), on one MI355X, beside the oracle ports
of the reference step() on one host core.

    python tools/facade_latency.py [--bg-episodes 100] [--sc-episodes 3]

* BeerGameEnv.step (beergame_env.py:66-138; reference ~12.8 us per step on one core,
  BASELINE.md §4): the facade writes the action into host-mapped memory and posts the week
  to its step server (a resident wave polling a host-mapped mailbox, scg_bg_server_step),
  which writes observation, reward and the overflow word to host-mapped memory; beside it the
  launch path (SCG_BG_SERVER=0: one step-kernel launch and one stream synchronisation per
  call) and the round-4 design (pinned H2D copy, launch, two D2H copies, synchronise), on the
  same box. The server's wave launches are counted. And 8 envs stepped round-robin (an SB3
  DummyVecEnv of drop-in envs): every env holds a slot of the one shared server, so the 8
  share one resident wave; per step() call, on the server and on the launch path.
* SupplyChain2perStageEnv.step (supplychain_env.py:703-748; reference ~136 us per step):
  its step server (a resident block of the node-parallel kernel polling a host-mapped
  mailbox, scg_sc_server_*) and the launch path (SCG_SC_SERVER=0), host RandomState episode
  draws (the reference's), float64 obs.
* cpu: oracle.beergame.BeerGameOracle.step and oracle.supplychain.SupplyChainOracle.step
  (the calibrated NumPy ports of the reference step, profiles/r04_cpu_calibration.json) on
  this box's host, one core.
Every timing is per step() call in wall-clock microseconds (median, 10th and 90th
percentile), reset() excluded. One JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)


def _stats(ts):
    import numpy as np
    a = np.asarray(ts) * 1e6
    return {"median_us": float(np.median(a)), "p10_us": float(np.percentile(a, 10)),
            "p90_us": float(np.percentile(a, 90)), "mean_us": float(a.mean()), "calls": int(a.size)}


def _time_episodes(env, actions, episodes, horizon):
    ts = []
    pc = time.perf_counter
    for e in range(episodes):
        env.reset()
        for w in range(horizon):
            a = actions[(e * horizon + w) % len(actions)]
            t0 = pc()
            env.step(a)
            ts.append(pc() - t0)
    return ts


def beergame(episodes, server=True):
    import numpy as np
    os.environ["SCG_BG_SERVER"] = "1" if server else "0"
    import gym_supplychain_amd as gsa
    env = gsa.make("beergame-v0")
    rng = np.random.RandomState(0)
    acts = [rng.randint(0, 9, size=4) for _ in range(35 * 8)]
    _time_episodes(env, acts, 2, 35)  # warm-up
    st = _stats(_time_episodes(env, acts, episodes, 35))
    if server:
        st["server_wave_launches"] = int(env._server.sv.launches)
    env.close()
    return st


def beergame_many(episodes, n_envs=8, server=True):
    import numpy as np
    os.environ["SCG_BG_SERVER"] = "1" if server else "0"
    import gym_supplychain_amd as gsa
    envs = [gsa.make("beergame-v0") for _ in range(n_envs)]
    rng = np.random.RandomState(0)
    acts = [rng.randint(0, 9, size=4) for _ in range(35 * 8)]
    pc = time.perf_counter

    def run(eps):
        ts = []
        for e in range(eps):
            for env in envs:
                env.reset()
            for w in range(35):
                a = acts[(e * 35 + w) % len(acts)]
                for env in envs:
                    t0 = pc()
                    env.step(a)
                    ts.append(pc() - t0)
        return ts
    run(2)
    l0 = envs[0]._server.sv.launches if server else 0
    st = _stats(run(episodes))
    st["n_envs"] = n_envs
    if server:
        st["servers"] = len({id(e._server.server) for e in envs})
        st["server_wave_launches"] = int(envs[0]._server.sv.launches - l0)
    for env in envs:
        env.close()
    return st


class _CopyingBeerGame:
    """The round-4 facade's step for comparison: pinned action row -> device copy, the step
    launch, obs/reward and overflow-word copies back, synchronise."""

    def __init__(self):
        import numpy as np
        import torch
        from gym_supplychain_amd import BeerGameVecEnv
        self.torch, self.np = torch, np
        self.vec = BeerGameVecEnv(1, {}, demand="fixed", auto_reset=False, track_costs=True, track_history=True,
                                  track_returns=False, full_table=True)
        self.act_host = torch.zeros((1, 4), dtype=torch.int32, pin_memory=True)
        self.act_dev = torch.zeros((1, 4), dtype=torch.int32, device=self.vec.device)
        self.out_host = torch.zeros(self.vec._out.shape, dtype=torch.int32, pin_memory=True)
        self.err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)

    def reset(self):
        self.vec.reset()

    def step(self, a):
        self.act_host.numpy()[0, :] = a
        self.act_dev.copy_(self.act_host, non_blocking=True)
        self.vec.step(self.act_dev)
        self.out_host.copy_(self.vec._out, non_blocking=True)
        self.err_host.copy_(self.vec._err, non_blocking=True)
        self.torch.cuda.current_stream(self.vec.device).synchronize()
        return self.out_host.numpy()[:4].astype(self.np.int64), self.np.int64(self.out_host.numpy()[4])


def beergame_copies(episodes):
    import numpy as np
    env = _CopyingBeerGame()
    rng = np.random.RandomState(0)
    acts = [rng.randint(0, 9, size=4) for _ in range(35 * 8)]
    _time_episodes(env, acts, 2, 35)
    return _stats(_time_episodes(env, acts, episodes, 35))


def supplychain(episodes, server=True):
    import numpy as np
    os.environ["SCG_SC_SERVER"] = "1" if server else "0"
    import gym_supplychain_amd as gsa
    env = gsa.make("sc-2perstage-v0", seed=0)
    rng = np.random.RandomState(0)
    acts = [rng.uniform(-1, 1, env.action_space.shape).astype(np.float32) for _ in range(720)]
    _time_episodes(env, acts, 1, 360)
    st = _stats(_time_episodes(env, acts, episodes, 360))
    if server:
        st["server_block_launches"] = env._server.launches
    env.close()
    return st, env._vec.kernel


def cpu_beergame(episodes):
    import numpy as np
    from oracle.beergame import BeerGameOracle
    env = BeerGameOracle({})
    rng = np.random.RandomState(0)
    acts = [rng.randint(0, 9, size=4) for _ in range(35 * 8)]
    _time_episodes(env, acts, 2, 35)
    return _stats(_time_episodes(env, acts, episodes, 35))


def cpu_supplychain(episodes):
    import numpy as np
    from gym_supplychain_amd.envs.scenarios import SCENARIOS as BUILDERS
    from oracle.sc_draws import sc_demand_table
    from oracle.supplychain import SupplyChainOracle
    nodes, kw = BUILDERS["sc-2perstage-v0"]()
    okw = {k: kw[k] for k in ("num_products", "unmet_demand_cost", "exceeded_stock_capacity_cost",
                              "exceeded_process_capacity_cost", "exceeded_ship_capacity_cost", "demand_range",
                              "processing_ratio", "stochastic_leadtimes", "avg_leadtime", "max_leadtime",
                              "total_time_steps")}
    o = SupplyChainOracle(nodes, **okw)
    T, R, P = okw["total_time_steps"], len(o.retailers), o.P
    rng = np.random.RandomState(0)
    acts = [rng.uniform(-1, 1, o.action_size).astype(np.float32) for _ in range(720)]

    class _Env:
        ep = 0

        def reset(self):
            o.reset(sc_demand_table(1, 0, self.ep, T, R, P, *okw["demand_range"]))
            self.ep += 1

        def step(self, a):
            return o.step(a)
    env = _Env()
    return _stats(_time_episodes(env, acts, episodes, T))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bg-episodes", type=int, default=100)
    ap.add_argument("--sc-episodes", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import torch
    dev = torch.cuda.get_device_name(0)

    def emit(what, ref_us, st, **kw):
        print(json.dumps({"measure": what, "device": dev, "reference_us_per_step": ref_us, **st, **kw}), flush=True)

    emit("BeerGameEnv.step (step server: resident wave, host-mapped mailbox and io)", 12.8, beergame(a.bg_episodes))
    emit("BeerGameEnv.step, launch path (SCG_BG_SERVER=0: host-mapped io, one launch + stream sync)", 12.8,
         beergame(a.bg_episodes, server=False))
    emit("BeerGameEnv.step, 8 envs round-robin (one shared step-server wave)", 12.8,
         beergame_many(max(a.bg_episodes // 8, 4)))
    emit("BeerGameEnv.step, 8 envs round-robin, launch path (SCG_BG_SERVER=0)", 12.8,
         beergame_many(max(a.bg_episodes // 8, 4), server=False))
    emit("BeerGameEnv.step, round-4 design (H2D copy, launch, 2 D2H copies, sync)", 12.8, beergame_copies(a.bg_episodes))
    st, kernel = supplychain(a.sc_episodes)
    emit("SupplyChain2perStageEnv.step (step server: resident block, host-mapped mailbox and io)", 136.0, st,
         kernel=kernel)
    st, kernel = supplychain(a.sc_episodes, server=False)
    emit("SupplyChain2perStageEnv.step, launch path (SCG_SC_SERVER=0: host-mapped io, one launch + stream sync)",
         136.0, st, kernel=kernel)
    if not a.no_cpu:
        emit("cpu: oracle.beergame.BeerGameOracle.step, one host core", 12.8, cpu_beergame(a.bg_episodes))
        emit("cpu: oracle.supplychain.SupplyChainOracle.step, one host core", 136.0, cpu_supplychain(a.sc_episodes))


if __name__ == "__main__":
    main()
