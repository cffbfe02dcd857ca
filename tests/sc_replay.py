"""Replay recorded sampled envs of a SupplyChain batch on the oracle (test helper).

A GPU test runs a full-size batch, records for a sample of envs the actions it fed, the
observations and rewards it got (the terminal observation at the episode's last step) and
the auto-reset observation; `replay` re-runs each sampled env on
oracle.supplychain.SupplyChainOracle with the same Philox demand / lead-time tables
(oracle/sc_draws.py) and reports every difference. Imports only NumPy and the oracle, so a
process pool can run envs in parallel without loading torch.
"""
import numpy as np

from oracle.sc_draws import sc_demand_table, sc_leadtime_table
from oracle.supplychain import SupplyChainOracle


def replay(job):
    """job = dict(env=global env id, nodes, okw (SupplyChainOracle kwargs), seed, R, n_lt,
    lt=(avg, max), demand_range, acts [K, A], obs [K, O], rew [K], reset_obs [O], T).
    Steps 1..T are episode 0; the obs recorded at step T is the terminal observation; the
    remaining K - T steps continue episode 1 from reset_obs. Returns a list of mismatches."""
    okw, T = job["okw"], job["T"]
    bad = []

    def oracle(ep):
        o = SupplyChainOracle(job["nodes"], **okw)
        dem = sc_demand_table(job["seed"], job["env"], ep, T, job["R"], okw["num_products"], *job["demand_range"])
        lts = None
        if okw.get("stochastic_leadtimes"):
            lts = sc_leadtime_table(job["seed"], job["env"], ep, T, job["n_lt"], *job["lt"])
        return o, o.reset(dem, lts)

    o, first = oracle(0)
    if not np.array_equal(first, job["first_obs"]):
        bad.append(("reset", 0))
    ret = 0.0
    for k in range(job["acts"].shape[0]):
        if k == T:
            o, obs1 = oracle(1)
            if not np.array_equal(obs1, job["reset_obs"]):
                bad.append(("autoreset obs", k))
        obs, r, done, _ = o.step(job["acts"][k].copy())
        ret = ret + r if k < T else ret
        if not np.array_equal(obs, job["obs"][k]):
            bad.append(("obs", k, int(np.flatnonzero(obs != job["obs"][k])[0])))
        if r != job["rew"][k]:
            bad.append(("reward", k, float(r), float(job["rew"][k])))
        if done != (k == T - 1):
            bad.append(("done", k))
        if len(bad) > 5:
            break
    if job.get("final_return") is not None and abs(ret - job["final_return"]) > 1e-9 * max(1.0, abs(ret)):
        bad.append(("final_return", ret, job["final_return"]))
    return job["env"], bad
