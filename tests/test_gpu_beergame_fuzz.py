"""Fuzz on the device: random BeerGame configurations (1-8 levels, 3-80 weeks, delays 0-70
with zeros mixed in, any initial inventory / pipeline / orders values, costs, per-env demand
tables, negative actions) through BeerGameVecEnv's step kernels (state slab and general,
ring and full shipment table), week by week against the oracle's batch restatement of
beergame_env.py:66-138 (oracle/beergame.py run_batch_episode), bit for bit."""
import numpy as np
import pytest
import torch

from oracle.beergame import run_batch_episode

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _config(seed):
    r = np.random.RandomState(500 + seed)
    L, T = int(r.randint(1, 9)), int(r.randint(3, 81))
    N = int(r.choice([64, 97, 256]))
    delays = r.randint(0, 5, size=T)
    long = r.rand(T) < 0.1
    delays[long] = r.randint(5, 71, size=int(long.sum()))
    info = dict(levels=L, shipment_delays=[int(d) for d in delays],
                initial_inventory=[int(x) for x in r.randint(-5, 40, size=L)],
                initial_shipment_value=int(r.randint(0, 12)), initial_orders_value=int(r.randint(0, 12)),
                inv_cost=int(r.randint(0, 6)), backlog_cost=int(r.randint(0, 6)))
    demand = r.randint(0, 41, size=(N, T)).astype(np.int64)
    actions = r.randint(-2, 21, size=(T, N, L)).astype(np.int64)
    return info, demand, actions


@pytest.mark.parametrize("variant", ["slab", "general", "full_table"])
@pytest.mark.parametrize("seed", list(range(20)))
def test_random_config_matches_oracle(seed, variant):
    from gym_supplychain_amd import BeerGameVecEnv
    info, demand, actions = _config(seed)
    T, N, L = actions.shape
    want = run_batch_episode(dict(info, customer_demand=demand[0].tolist()), demand, actions)
    kw = dict(state_slab=variant == "slab", full_table=variant == "full_table")
    env = BeerGameVecEnv(N, dict(info, customer_demand=demand[0].tolist()),
                         demand=torch.as_tensor(demand.T.copy(), dtype=torch.int32, device=DEV), device=DEV,
                         auto_reset=False, track_history=True, **kw)
    obs = env.reset()
    assert np.array_equal(obs.cpu().numpy(), want["reset_obs"]), (seed, variant)
    acts = torch.as_tensor(actions, dtype=torch.int32, device=DEV)
    for w in range(T):
        obs, rew, done, _ = env.step(acts[w])
        assert np.array_equal(obs.cpu().numpy(), want["obs"][w]), (seed, variant, w)
        assert np.array_equal(rew.cpu().numpy(), want["reward"][w]), (seed, variant, w)
        assert np.array_equal(env.inventory.cpu().numpy(), want["inventory"][w]), (seed, variant, w)
        assert np.array_equal(env.backlog.cpu().numpy(), want["backlog"][w]), (seed, variant, w)
        assert np.array_equal(env.orders_placed.cpu().numpy(), want["orders_placed"][w]), (seed, variant, w)
        assert bool(done.all()) == (w == T - 1)
    assert np.array_equal(env.inventory_costs.cpu().numpy(), want["inventory_costs"])
    assert np.array_equal(env.backlog_costs.cpu().numpy(), want["backlog_costs"])
    assert np.array_equal(env.all_orders_placed.cpu().numpy(), want["all_orders_placed"])
    env.check_errors()
