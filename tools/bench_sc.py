"""SupplyChain throughput (BASELINE configs 3 and 4) — one JSON line per scenario.

    python tools/bench_sc.py [--scenario 2perstage|ntom|both] [--steps K] [--warmup W]

config 3: sc-2perstage-v0 defaults, 65,536 envs (8 nodes, 1 product, 14 actions, 27 obs)
config 4: ntom = SupplyChainNPerStage([8, 8, 8, 16]) defaults (2 products), 262,144 envs
          (40 nodes, 528 actions, 273 obs)
A step = one SupplyChainVecEnv.step() over the batch (one sc_step_kernel launch), float32
actions U[-1, 1] pre-generated on device (a pool cycled over the timed steps), float32
observations, auto-reset at the horizon. Kernel time from torch.cuda.Events around each
launch on the launch stream. `roofline.achieved` uses SURVEY §8(d)'s algorithmic bytes per
env-step (2 x state + actions + observation + reward + demand: 1,148 B for config 3 and
36,108 B for config 4). The CPU baseline times oracle.supplychain.SupplyChainOracle (the
NumPy restatement of the reference step) on the host cores.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0
SCENARIOS = {
    "2perstage": dict(env_id="sc-2perstage-v0", kwargs={}, n_envs=65536, bytes_per_env_step=1148,
                      baseline_cfg="configs[2]"),
    # not a BASELINE config: the two-product 2-per-stage chain (4 registered ids), whose
    # node-parallel block needs a whole CU's LDS; SURVEY §8(d)'s formula with H = 4:
    # 2 x 16 x (8 + 4 x 12 + 4) + 28 x 4 + 53 x 4 + 8 + 2 x 2 x 8
    "2perstage_mp": dict(env_id="sc-2perstage-multiproduct-v0", kwargs={}, n_envs=65536, bytes_per_env_step=2284,
                         baseline_cfg="none; 2-product sc-2perstage"),
    "ntom": dict(env_id="sc-Nperstage-multiproduct-v0", kwargs=dict(nodes_per_echelon=[8, 8, 8, 16]),
                 n_envs=262144, bytes_per_env_step=36108, baseline_cfg="configs[3]"),
}


def _cpu_worker(name, idx, budget, start):
    import numpy as np
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
    from gym_supplychain_amd.envs.scenarios import SCENARIOS as BUILDERS  # config only, no GPU use
    from oracle.sc_draws import sc_demand_table
    from oracle.supplychain import SupplyChainOracle
    sc = SCENARIOS[name]
    nodes, kw = BUILDERS[sc["env_id"]](**sc["kwargs"])
    okw = {k: kw[k] for k in ("num_products", "unmet_demand_cost", "exceeded_stock_capacity_cost",
                              "exceeded_process_capacity_cost", "exceeded_ship_capacity_cost", "demand_range",
                              "processing_ratio", "stochastic_leadtimes", "avg_leadtime", "max_leadtime",
                              "total_time_steps")}
    o = SupplyChainOracle(nodes, **okw)
    T, R, P = okw["total_time_steps"], len(o.retailers), o.P
    rng = np.random.RandomState(idx)
    start()  # every worker's chain is built: the timed parts start together
    steps, ep = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget:
        o.reset(sc_demand_table(1, idx, ep, T, R, P, *okw["demand_range"]))
        for _ in range(T):
            o.step(rng.uniform(-1, 1, o.action_size).astype(np.float32))
            steps += 1
            if time.perf_counter() - t0 >= budget:
                break
        ep += 1
    return steps, time.perf_counter() - t0


def cpu_baseline(name, budget=2.5):
    """SupplyChainOracle on every core of the affinity mask (bench.host_cpus / cpu_pool)."""
    import functools

    from bench import cpu_note, cpu_pool, host_cpus
    cpus = host_cpus()
    procs = cpus["procs"]
    value, steps = cpu_pool(functools.partial(_cpu_worker, name), budget, procs)
    return {"value": value, "unit": "env-steps/s", "cores": procs, "kind": "port", **cpus, "budget_s": budget,
            "sample": f"{procs} processes ({cpu_note(cpus)}) x {budget} s of "
                      f"{SCENARIOS[name]['env_id']} steps, one env per process, timed parts started together, "
                      f"oracle.supplychain.SupplyChainOracle; {steps} env-steps"}


def pmc_traffic(symbol, n_envs, name, kernel, build_info):
    """HBM bytes per launch of `symbol` from the newest committed PMC summary of exactly this
    workload — scenario, batch size, kernel choice and ledger mode — collected on this
    tree's SupplyChain sources (bench.pmc_lookup; tools/gpu_sc_traffic.sh writes them)."""
    from bench import pmc_lookup
    workload = {"bench": "bench_sc", "scenario": name, "n_envs": n_envs, "kernel": kernel, "build_info": bool(build_info)}
    return pmc_lookup("sc", workload, symbol.split("::")[-1])


def run(name, steps, warmup, n_envs, cpu, kernel="auto", build_info=False):
    import torch
    import gym_supplychain_amd as gsa
    sc = SCENARIOS[name]
    N = n_envs or sc["n_envs"]
    dev = torch.device("cuda", 0)
    env = gsa.make_vec(sc["env_id"], N, seed=0, device=dev, obs_dtype=torch.float32, auto_reset=True, kernel=kernel,
                       build_info=build_info, **sc["kwargs"])
    gen = torch.Generator(device=dev).manual_seed(0)
    pool = [torch.rand((N, env.n_actions), generator=gen, device=dev) * 2 - 1 for _ in range(4)]
    env.reset()
    for i in range(warmup):
        env.step(pool[i % 4])
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record(stream)
        env.step(pool[i % 4])
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if not os.environ.get("SCG_BENCH_NO_CHECK"):  # timing-only ablation builds break the dynamics
        env.check_errors()
    kern_s = sum(s.elapsed_time(e) for s, e in ev) / 1e3 / steps
    bpe = sc["bytes_per_env_step"]
    achieved = bpe * N / kern_s / 1e9
    traffic, traffic_src = pmc_traffic(env.kernel_symbol, N, name, kernel, build_info)
    line = {"metric": f"env-steps/sec, {sc['env_id']} {sc['kwargs'] or ''} x{N} envs on 1 MI355X",
            "value": N * steps / wall, "unit": "env-steps/s", "n_gpus": 1, "steps": steps, "warmup": warmup,
            "ms_per_step": wall * 1e3 / steps, "higher_is_better": True, "dtype": "f32 actions/obs, f64 state",
            "data": "synthetic: uniform demand drawn on device (Philox4x32-10), U[-1,1] float32 actions",
            "config": {"workload": f"{sc['env_id']} step() (BASELINE {sc['baseline_cfg']})", "n_envs": N,
                       "kernel": env.kernel,
                       "n_actions": env.n_actions, "n_obs": env.n_obs, "heap_capacity": env.heap_capacity,
                       "build_info": build_info},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": bpe * N, "kernel": env.kernel_symbol,
                         "avg_kernel_us": kern_s * 1e6, "bytes_per_env_step": bpe}}
    del env, pool
    torch.cuda.empty_cache()
    if cpu:
        line["cpu_baseline"] = cpu_baseline(name)
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="both", choices=["2perstage", "2perstage_mp", "ntom", "both", "all"])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--envs", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel", default="auto", choices=["auto", "lane", "level", "staged", "nodes", "all", "both"])
    ap.add_argument("--build-info", action="store_true", help="keep the build_info ledgers (info['sc_episode'])")
    ap.add_argument("--nodes-max-blocks", type=int, default=0,
                    help="cap the node-parallel kernel's persistent grid (scg_sc_nodes_max_blocks; experiments)")
    a = ap.parse_args()
    if a.nodes_max_blocks:
        from gym_supplychain_amd import _native as nat
        nat.lib.scg_sc_nodes_max_blocks(a.nodes_max_blocks)
    names = {"both": ["2perstage", "ntom"], "all": ["2perstage", "2perstage_mp", "ntom"]}.get(a.scenario, [a.scenario])
    for name in names:
        kernels = [a.kernel]
        if a.kernel in ("all", "both"):  # the node-parallel kernel only takes chains whose block fits LDS
            kernels = ["lane", "level", "staged"] + (["nodes"] if name != "ntom" else [])
        for k in kernels:
            run(name, a.steps, a.warmup, a.envs, not a.no_cpu_baseline and k == kernels[-1], k, a.build_info)


if __name__ == "__main__":
    main()
