"""GPU parity of the SupplyChain kernels (through the C ABI) with the reference's golden
vectors (observations, rewards, stocks, heap storage order — bit-exact in float64) and,
at BASELINE sizes, with the oracle on sampled envs of the full batch."""
import numpy as np
import pytest
import torch

from golden_io import load_sc, sc_cases
from oracle.sc_draws import sc_demand_table, sc_leadtime_table
from oracle.supplychain import SupplyChainOracle

pytestmark = pytest.mark.gpu
CASES = sc_cases()
DEV = "cuda"
KERNELS = ["lane", "level", "staged", "nodes"]


def _or_skip(make, kernel):
    """make(), skipping when the node-parallel kernel cannot take the chain (its block's
    heaps and inbox must fit LDS; scg_sc_prepare rejects it otherwise)."""
    try:
        return make()
    except ValueError as e:
        if kernel == "nodes" and "node-parallel" in str(e):
            pytest.skip(f"chain too wide for the node-parallel kernel: {e}")
        raise


def _vec(meta, n, **kw):
    from gym_supplychain_amd import SupplyChainVecEnv
    ekw = dict(meta["kwargs"])
    ekw.pop("seed", None)
    kw.setdefault("seed", meta["seed"])
    ekw.update(kw)
    return SupplyChainVecEnv(n, meta["nodes_info"], device=DEV, **ekw)


def _check_heaps(env, g, t, n, name):
    heaps = env.heaps(n)
    for i, node in enumerate(heaps):
        for p, h in enumerate(node):
            k = int((g["heap_t"][t, n, i, p] >= 0).sum())
            assert [x[0] for x in h] == g["heap_t"][t, n, i, p, :k].tolist(), (name, t, n, i, p)
            assert [x[1] for x in h] == g["heap_v"][t, n, i, p, :k].tolist(), (name, t, n, i, p)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", CASES)
def test_step_matches_reference(name, kernel):
    g = load_sc(name)
    meta = g["meta"]
    T, N = meta["T"], g["obs"].shape[1]
    env = _or_skip(lambda: _vec(meta, N, obs_dtype=torch.float64, auto_reset=False, kernel=kernel), kernel)
    assert env.kernel == kernel
    dem, lts = env.draw_tables(0)
    assert np.array_equal(dem.cpu().numpy(), g["demands"])
    if meta["n_lt"]:
        assert np.array_equal(lts.cpu().numpy(), g["leadtimes"])
    obs = env.reset()
    assert np.array_equal(obs.cpu().numpy(), g["obs"][0])
    acts = torch.as_tensor(g["actions"], device=DEV)
    heap_check_steps = {0, 1, 2, T // 2, T - 1, T}
    for t in range(T):
        obs, rew, done, info = env.step(acts[t])
        assert np.array_equal(obs.cpu().numpy(), g["obs"][t + 1]), (name, t)
        assert np.array_equal(rew.cpu().numpy(), g["reward"][t]), (name, t)
        assert np.array_equal(env.stock.cpu().numpy(), g["stock"][t + 1]), (name, t)
        assert bool(done.all()) == (t == T - 1)
        if t + 1 in heap_check_steps:
            for n in range(N):
                _check_heaps(env, g, t + 1, n, name)
    assert np.allclose(env.final_return.cpu().numpy(), g["reward"].sum(0), rtol=1e-12, atol=0)
    env.check_errors()
    with pytest.raises(IndexError):
        env.step(acts[0])


@pytest.mark.parametrize("name", CASES)
def test_nodes_kernel_serial_walk_matches_reference(name):
    """The node-parallel kernel's path for envs whose receive order it cannot prove
    (sc_nodes_serial: the nodes one after another on the staged heaps), forced for every
    env with SCG_SC_SERIAL, against the reference's golden vectors."""
    from gym_supplychain_amd import _native as nat
    g = load_sc(name)
    meta = g["meta"]
    T, N = meta["T"], g["obs"].shape[1]
    env = _or_skip(lambda: _vec(meta, N, obs_dtype=torch.float64, auto_reset=False, kernel="nodes"), "nodes")
    env._flags |= nat.SCG_SC_SERIAL
    env.reset()
    acts = torch.as_tensor(g["actions"], device=DEV)
    for t in range(T):
        obs, rew, _, _ = env.step(acts[t])
        assert np.array_equal(obs.cpu().numpy(), g["obs"][t + 1]), (name, t)
        assert np.array_equal(rew.cpu().numpy(), g["reward"][t]), (name, t)
        assert np.array_equal(env.stock.cpu().numpy(), g["stock"][t + 1]), (name, t)
    for n in range(N):
        _check_heaps(env, g, T, n, name)
    env.check_errors()


@pytest.mark.parametrize("name", ["2perstage", "2perstage_stoch"])
def test_float32_observations(name):
    g = load_sc(name)
    meta = g["meta"]
    T, N = meta["T"], g["obs"].shape[1]
    env = _vec(meta, N, obs_dtype=torch.float32, auto_reset=False)
    obs = env.reset()
    assert np.array_equal(obs.cpu().numpy(), g["obs"][0].astype(np.float32))
    acts = torch.as_tensor(g["actions"], device=DEV)
    for t in range(T):
        obs, rew, _, _ = env.step(acts[t])
        assert np.array_equal(obs.cpu().numpy(), g["obs"][t + 1].astype(np.float32))
        assert np.array_equal(rew.cpu().numpy(), g["reward"][t])


def test_single_env_facade_and_reference_known_answers():
    """The reference's hand-traced test (test_supplychain_2perstage_env.py:28-170) through
    the drop-in class, with its RandomState(0) demand replayed via a demand table."""
    from gym_supplychain_amd import SupplyChainVecEnv
    from gym_supplychain_amd.envs.scenarios import two_per_stage_nodes
    from test_oracle_supplychain import KA_ACTIONS, KA_OBS, KA_RESET_OBS, KA_REWARDS
    nodes, kw = two_per_stage_nodes(total_time_steps=5, ship_capacity=250)
    kw.pop("seed")
    dem = np.random.RandomState(0).randint(10, 21, size=(1, 6, 2, 1))
    env = SupplyChainVecEnv(1, nodes, device=DEV, obs_dtype=torch.float64, auto_reset=False,
                            demand_table=torch.as_tensor(dem, dtype=torch.int32, device=DEV), **kw)
    assert np.allclose(env.reset().cpu().numpy()[0], KA_RESET_OBS)
    for act, want_obs, want_r in zip(KA_ACTIONS, KA_OBS, KA_REWARDS):
        a = torch.as_tensor(2 * np.array(act, dtype=np.float32) - 1, device=DEV).reshape(1, -1)
        obs, r, _, _ = env.step(a)
        assert np.allclose(obs.cpu().numpy()[0], want_obs)
        assert np.round(float(r[0]), 3) == want_r

    from gym_supplychain_amd import SupplyChain2perStageEnv
    e = SupplyChain2perStageEnv(total_time_steps=5, seed=3)
    o = e.reset()
    assert o.dtype == np.float64 and o.shape == (27,) and e.action_space.shape == (14,)
    obs, r, done, info = e.step(np.zeros(14, dtype=np.float32))
    assert obs.dtype == np.float64 and isinstance(r, np.float64) and info == {} and done is False
    for _ in range(4):
        obs, r, done, info = e.step(np.zeros(14, dtype=np.float32))
    assert done is True
    with pytest.raises(IndexError):
        e.step(np.zeros(14, dtype=np.float32))


@pytest.mark.parametrize("kernel", ["lane", "staged"])
def test_single_env_kernel_choice_gives_the_same_episode(kernel):
    """The drop-in env takes the node-parallel kernel by default (a latency choice, not the
    batch occupancy rule); an explicitly named kernel runs the same episode: observations,
    rewards and done, bit for bit, with the reference's host RandomState draws."""
    from gym_supplychain_amd import SupplyChainEnv
    from gym_supplychain_amd.envs.scenarios import two_per_stage_nodes
    nodes, kw = two_per_stage_nodes(total_time_steps=40)
    kw.pop("seed", None)
    a = SupplyChainEnv(nodes, seed=11, device=DEV, **kw)
    b = SupplyChainEnv(nodes, seed=11, device=DEV, kernel=kernel, **kw)
    assert a._vec.kernel == "nodes" and b._vec.kernel == kernel
    rng = np.random.RandomState(3)
    for ep in range(2):
        assert np.array_equal(a.reset(), b.reset())
        done = False
        while not done:
            act = rng.uniform(-1, 1, a.action_space.shape).astype(np.float32)
            o1, r1, done, _ = a.step(act)
            o2, r2, d2, _ = b.step(act)
            assert np.array_equal(o1, o2) and r1 == r2 and done == d2


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("scenario,n_envs,steps", [("sc-2perstage-v0", 65536, 6),
                                                   ("sc-Nperstage-multiproduct-v0", 262144, 2)])
def test_full_size_sampled_envs_match_oracle(scenario, n_envs, steps, kernel):
    """BASELINE configs 3 and 4 at full size; every step checks 8 sampled envs of the
    batch against the oracle (envs are independent, so a sample checks the full launch)."""
    import gym_supplychain_amd as gsa
    kw = {} if scenario == "sc-2perstage-v0" else dict(nodes_per_echelon=[8, 8, 8, 16])
    seed = 77
    env = _or_skip(lambda: gsa.make_vec(scenario, n_envs, seed=seed, device=DEV, obs_dtype=torch.float64,
                                        auto_reset=False, kernel=kernel, **kw), kernel)
    sp = env.spec
    nodes_info = (gsa.envs.scenarios.SCENARIOS[scenario](**kw))[0]
    okw = dict(num_products=sp.P, demand_range=sp.demand_range, processing_ratio=sp.processing_ratio,
               stochastic_leadtimes=sp.stochastic_leadtimes, avg_leadtime=sp.avg_leadtime,
               max_leadtime=sp.max_leadtime, total_time_steps=sp.total_time_steps, **sp.penalties)
    sample = [0, 1, 63, 64, 4097, n_envs // 2 + 5, n_envs - 2, n_envs - 1]
    oracles = []
    obs = env.reset().cpu().numpy()
    for n in sample:
        o = SupplyChainOracle(nodes_info, **okw)
        dem = sc_demand_table(seed, n, 0, sp.total_time_steps, sp.n_retailers, sp.P, *sp.demand_range)
        assert np.array_equal(o.reset(dem), obs[n])
        oracles.append(o)
    gen = torch.Generator(device=DEV).manual_seed(5)
    for t in range(steps):
        a = torch.rand((n_envs, env.n_actions), generator=gen, device=DEV, dtype=torch.float32) * 2 - 1
        obs, rew, _, _ = env.step(a)
        a_np, obs_np, rew_np = a.cpu().numpy(), obs.cpu().numpy(), rew.cpu().numpy()
        for n, o in zip(sample, oracles):
            want_obs, want_r, _, _ = o.step(a_np[n].copy())
            assert np.array_equal(obs_np[n], want_obs), (scenario, t, n)
            assert rew_np[n] == want_r, (scenario, t, n)
    env.check_errors()


@pytest.mark.parametrize("kernel", KERNELS)
def test_autoreset_and_stochastic_episodes_match_oracle(kernel):
    from gym_supplychain_amd import SupplyChainVecEnv
    from gym_supplychain_amd.envs.scenarios import two_per_stage_nodes
    nodes, kw = two_per_stage_nodes(total_time_steps=7, stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4)
    kw.pop("seed")
    N, seed = 1000, 4242
    env = SupplyChainVecEnv(N, nodes, seed=seed, device=DEV, obs_dtype=torch.float64, auto_reset=True,
                            kernel=kernel, **kw)
    sp = env.spec
    okw = dict(num_products=sp.P, demand_range=sp.demand_range, processing_ratio=sp.processing_ratio,
               stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4, total_time_steps=7, **sp.penalties)
    sample = [0, 17, 999]
    obs = env.reset().cpu().numpy()
    gen = torch.Generator(device=DEV).manual_seed(9)
    for ep in range(3):
        oracles = []
        for n in sample:
            o = SupplyChainOracle(nodes, **okw)
            dem = sc_demand_table(seed, n, ep, 7, sp.n_retailers, sp.P, *sp.demand_range)
            lts = sc_leadtime_table(seed, n, ep, 7, sp.n_leadtimes, 2, 4)
            assert np.array_equal(o.reset(dem, lts), obs[n])
            oracles.append(o)
        for t in range(7):
            a = torch.rand((N, env.n_actions), generator=gen, device=DEV) * 2.2 - 1.1
            obs_t, rew, done, info = env.step(a)
            a_np, rew_np = a.cpu().numpy(), rew.cpu().numpy()
            shown = (info["terminal_observation"] if t == 6 else obs_t).cpu().numpy()
            for n, o in zip(sample, oracles):
                want_obs, want_r, want_done, _ = o.step(a_np[n].copy())
                assert np.array_equal(shown[n], want_obs), (ep, t, n)
                assert rew_np[n] == want_r
            assert bool(done.all()) == (t == 6)
            if t == 6:
                for n, o in zip(sample, oracles):
                    assert info["episode_return"][n].item() == pytest.approx(o.episode_rewards, rel=1e-12)
        obs = obs_t.cpu().numpy()
        assert env.episode == ep + 1 and env.time_step == 0
    env.check_errors()


def test_sharding_is_invariant():
    from gym_supplychain_amd import SupplyChainVecEnv
    from gym_supplychain_amd.envs.scenarios import two_per_stage_nodes
    nodes, kw = two_per_stage_nodes(total_time_steps=10)
    kw.pop("seed")
    N = 512
    whole = SupplyChainVecEnv(N, nodes, seed=8, device=DEV, **kw)
    parts = [SupplyChainVecEnv(N // 2, nodes, seed=8, env_offset=o, device=DEV, **kw) for o in (0, N // 2)]
    whole.reset()
    for p in parts:
        p.reset()
    gen = torch.Generator(device=DEV).manual_seed(1)
    for t in range(10):
        a = torch.rand((N, whole.n_actions), generator=gen, device=DEV) * 2 - 1
        o, r, _, _ = whole.step(a)
        o1, r1, _, _ = parts[0].step(a[: N // 2])
        o2, r2, _, _ = parts[1].step(a[N // 2:])
        assert torch.equal(o, torch.cat([o1, o2])) and torch.equal(r, torch.cat([r1, r2]))


@pytest.mark.parametrize("scenario,kw", [("sc-2perstage-v0", dict(total_time_steps=12, stochastic_leadtimes=True,
                                                                  avg_leadtime=2, max_leadtime=4)),
                                         ("sc-Nperstage-multiproduct-v0", dict(nodes_per_echelon=[3, 5, 2, 7],
                                                                              num_products=3, total_time_steps=9))])
def test_level_kernel_equals_lane_kernel(scenario, kw):
    """Both kernels over every env of a batch, two episodes with auto-reset, ragged level
    widths (3, 5, 2, 7) and a tail block: identical obs, rewards, returns and stocks."""
    import gym_supplychain_amd as gsa
    N = 3001
    envs = []
    for k in KERNELS:
        try:
            envs.append(gsa.make_vec(scenario, N, seed=21, device=DEV, obs_dtype=torch.float64, kernel=k, **kw))
        except ValueError as e:  # the node-parallel kernel only takes chains whose block fits LDS
            assert k == "nodes" and "node-parallel" in str(e)
    assert [e.kernel for e in envs] == KERNELS[:len(envs)]
    o = [e.reset() for e in envs]
    assert torch.equal(o[0], o[1])
    gen = torch.Generator(device=DEV).manual_seed(3)
    T = envs[0].spec.total_time_steps
    for t in range(2 * T):
        a = torch.rand((N, envs[0].n_actions), generator=gen, device=DEV) * 2.4 - 1.2
        (o0, r0, d0, i0), *rest = (e.step(a) for e in envs)
        for e, (o1, r1, d1, i1) in zip(envs[1:], rest):
            assert torch.equal(o0, o1) and torch.equal(r0, r1) and torch.equal(d0, d1), (t, e.kernel)
            assert torch.equal(envs[0].stock, e.stock), (t, e.kernel)
            if i0:
                assert torch.equal(i0["terminal_observation"], i1["terminal_observation"])
                assert torch.equal(i0["episode_return"], i1["episode_return"])
    for e in envs:
        e.check_errors()


@pytest.mark.parametrize("max_blocks", [2, 3, 0])
@pytest.mark.parametrize("n_envs", [324, 322])
@pytest.mark.parametrize("scenario,kw", [
    ("sc-2perstage-v0", dict(total_time_steps=12, stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4)),
    ("sc-2perstage-multiproduct-v0", dict(total_time_steps=9, build_info=True, obs_dtype=torch.float32)),
    ("sc-2perstage-v0", dict(total_time_steps=7, serial=True))])
def test_nodes_kernel_persistent_tiles_equal_lane_kernel(scenario, kw, n_envs, max_blocks):
    """The node-parallel kernel's persistent grid (scg_sc_nodes_max_blocks caps it, so a
    block steps several 64-env tiles in turn) against the lane kernel over every env, two
    episodes with auto-reset, with a 4- or 2-env tail tile; stochastic lead times, two
    products with ledgers, and every env on the serial walk — identical obs, rewards,
    returns, stocks, heaps and ledgers. The cap applies to the ledger instantiation too, so
    with max_blocks 2 or 3 this test deliberately runs its tile loop over several tiles per
    block, which production never does (that instantiation keeps one block per tile,
    SCG_NODES_LED_PERSISTENT=0); max_blocks 0 is the production grid."""
    import gym_supplychain_amd as gsa
    from gym_supplychain_amd import _native as nat
    kw = dict(kw)
    serial = kw.pop("serial", False)
    kw.setdefault("obs_dtype", torch.float64)  # the two-product block fits LDS with float32 observations
    envs = [gsa.make_vec(scenario, n_envs, seed=5, device=DEV, kernel=k, **kw)
            for k in ("lane", "nodes")]
    assert envs[1].kernel == "nodes"
    if serial:
        envs[1]._flags |= nat.SCG_SC_SERIAL
    prev = nat.lib.scg_sc_nodes_max_blocks(max_blocks)
    try:
        o = [e.reset() for e in envs]
        assert torch.equal(o[0], o[1])
        gen = torch.Generator(device=DEV).manual_seed(11)
        T = envs[0].spec.total_time_steps
        for t in range(2 * T):
            a = torch.rand((n_envs, envs[0].n_actions), generator=gen, device=DEV) * 2.4 - 1.2
            (o0, r0, d0, i0), (o1, r1, d1, i1) = (e.step(a) for e in envs)
            assert torch.equal(o0, o1) and torch.equal(r0, r1) and torch.equal(d0, d1), t
            assert torch.equal(envs[0].stock, envs[1].stock), t
            assert torch.equal(envs[0]._heap_size, envs[1]._heap_size), t  # both env-fastest
            if envs[0].build_info:
                assert torch.equal(envs[0]._led, envs[1]._led) and torch.equal(envs[0]._led_k, envs[1]._led_k), t
            if "terminal_observation" in i0:
                assert torch.equal(i0["terminal_observation"], i1["terminal_observation"])
                assert torch.equal(i0["episode_return"], i1["episode_return"])
        for n in (0, 100, n_envs - 1):
            assert envs[0].heaps(n) == envs[1].heaps(n)
    finally:
        nat.lib.scg_sc_nodes_max_blocks(prev)
    for e in envs:
        e.check_errors()


@pytest.mark.parametrize("kernel", ["lane", "staged", "nodes"])
@pytest.mark.parametrize("name", CASES)
def test_ledgers_match_reference(name, kernel):
    """build_info: info['sc_episode'] on the device against the reference's ledgers after
    every step — values and NumPy types of every cost/unit entry, exactly (every kernel
    that keeps ledgers; the node-parallel one where its LDS takes the chain)."""
    from gym_supplychain_amd import _native as nat
    g = load_sc(name)
    meta = g["meta"]
    T, N = meta["T"], g["obs"].shape[1]
    env = _or_skip(lambda: _vec(meta, N, obs_dtype=torch.float64, auto_reset=False, build_info=True, kernel=kernel),
                   kernel)
    assert env.kernel == kernel
    env.reset()
    acts = torch.as_tensor(g["actions"], device=DEV)
    for t in range(T):
        _, rew, _, info = env.step(acts[t])
        led = info["sc_episode"]
        for j, key in enumerate(nat.SC_LEDGER_NAMES):
            assert np.array_equal(led["costs"][key].cpu().numpy(), g["led_cost"][t, :, j]), (name, t, key)
            assert np.array_equal(led["units"][key].cpu().numpy(), g["led_units"][t, :, j]), (name, t, key)
        k = env.ledger_kinds().cpu().numpy()                       # [2, 8, P, N]
        assert np.array_equal(k[0].transpose(2, 0, 1), g["led_cost_k"][t]), (name, t)
        assert np.array_equal(k[1].transpose(2, 0, 1), g["led_units_k"][t]), (name, t)
        assert np.allclose(led["rewards"].cpu().numpy(), g["led_rewards"][t], rtol=1e-12, atol=0)
    env.check_errors()


def test_ledgers_autoreset_and_reference_known_answers():
    """Terminal-step ledger kept across auto-reset; the reference's own ledger tests
    (test_multiproduct.py:123-237) through the drop-in types."""
    from gym_supplychain_amd import SupplyChainVecEnv
    from test_oracle_supplychain import KA_LEDGERS, ka_multiproduct_chain
    nodes, kw = ka_multiproduct_chain()
    for case, (T, acts, want) in sorted(KA_LEDGERS.items()):
        dem = np.random.RandomState(0).randint(0, 6, size=(1, T + 1, 1, 2))
        env = SupplyChainVecEnv(1, nodes, device=DEV, obs_dtype=torch.float64, auto_reset=False, build_info=True,
                                total_time_steps=T, demand_table=torch.as_tensor(dem, dtype=torch.int32, device=DEV),
                                **kw)
        env.reset()
        for a in acts:
            env.step(torch.as_tensor(2 * np.array(a, dtype=np.float32) - 1, device=DEV).reshape(1, -1))
        got = env.sc_episode(0)
        for key, (units, costs) in want.items():
            assert got["units"][key] == units and got["costs"][key] == costs, (case, key)
    # auto-reset: 2 episodes of 7 steps, oracle ledgers at every terminal step
    from gym_supplychain_amd.envs.scenarios import two_per_stage_nodes
    nodes, kw = two_per_stage_nodes(total_time_steps=7, build_info=True)
    kw.pop("seed")
    N, seed = 300, 99
    env = SupplyChainVecEnv(N, nodes, seed=seed, device=DEV, obs_dtype=torch.float64, auto_reset=True, **kw)
    sp = env.spec
    okw = dict(num_products=sp.P, demand_range=sp.demand_range, processing_ratio=sp.processing_ratio,
               total_time_steps=7, **sp.penalties)
    env.reset()
    gen = torch.Generator(device=DEV).manual_seed(4)
    for ep in range(2):
        oracles = []
        for n in (0, 150, 299):
            o = SupplyChainOracle(nodes, build_info=True, **okw)
            o.reset(sc_demand_table(seed, n, ep, 7, sp.n_retailers, sp.P, *sp.demand_range))
            oracles.append((n, o))
        for t in range(7):
            a = torch.rand((N, env.n_actions), generator=gen, device=DEV) * 2 - 1
            _, _, _, info = env.step(a)
            a_np = a.cpu().numpy()
            for n, o in oracles:
                _, _, _, oinfo = o.step(a_np[n].copy())
            if t < 6:
                assert "terminal_sc_episode" not in info
        for n, o in oracles:
            got = env.sc_episode(n, final=True)
            want = o.est_episode
            assert got["costs"] == want["costs"] and got["units"] == want["units"], (ep, n)
            assert [type(x) for x in got["costs"]["ship"]] == [type(x) for x in want["costs"]["ship"]]
            assert got["rewards"] == pytest.approx(float(want["rewards"]), rel=1e-12)
        assert all(float(x) == 0 for x in env.sc_episode(0)["costs"]["stock"])   # fresh episode


def test_drop_in_env_build_info():
    """The drop-in class with build_info=True: info['sc_episode'] every step, one dict per
    episode mutated in place, costs summing to -rewards (the reference's check_rewards,
    tests/utils.py:3-12)."""
    from gym_supplychain_amd import SupplyChain2perStageEnv
    e = SupplyChain2perStageEnv(total_time_steps=6, seed=5, build_info=True)
    e.reset()
    rng = np.random.RandomState(0)
    total, first = 0.0, None
    for t in range(6):
        _, r, done, info = e.step(rng.uniform(-1, 1, 14).astype(np.float32))
        total += r
        led = info["sc_episode"]
        first = led if first is None else first
        assert led is first and isinstance(led["rewards"], np.float64)
        assert np.isclose(led["rewards"], total)
        assert np.isclose(total, -sum(float(x) for k in led["costs"] for x in led["costs"][k]))
    assert done


def test_auto_kernel_symbols():
    """kernel='auto' on the bench configs: the node-parallel kernel (config 3), the
    node-staged kernel (config 4); kernel_symbol names what rocprofv3 reports."""
    import gym_supplychain_amd as gsa
    env = gsa.make_vec("sc-2perstage-v0", 64, device=DEV)
    assert env.kernel == "nodes" and env.kernel_symbol == "scg::sc_step_nodes_kernel<2, false, false>"
    env = gsa.make_vec("sc-2perstage-v0", 64, device=DEV, build_info=True)
    assert env.kernel == "nodes" and env.kernel_symbol == "scg::sc_step_nodes_kernel<2, false, true>"
    env = gsa.make_vec("sc-2perstage-v0", 64, device=DEV, kernel="lane")
    assert env.kernel == "lane" and env.kernel_symbol == "scg::sc_step_lds_kernel<2, 32>"
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    env = gsa.make_vec("sc-2perstage-v0", cus * 512, device=DEV, kernel="lane")
    assert env.kernel_symbol == "scg::sc_step_lds_kernel<2, 64>"
    env = gsa.make_vec("sc-2perstage-multiproduct-v0", 64, device=DEV)  # one block per CU
    assert env.kernel == "nodes" and env.kernel_symbol == "scg::sc_step_nodes_kernel<2, false, false>"
    env = gsa.make_vec("sc-Nperstage-multiproduct-v0", 64, device=DEV, nodes_per_echelon=[8, 8, 8, 16])
    assert env.kernel == "staged" and env.kernel_symbol == "scg::sc_step_staged_kernel<16, false>"
    env = gsa.make_vec("sc-2perstage-v0", 64, device=DEV, kernel="level")
    assert env.kernel_symbol.startswith("scg::sc_level_kernel<2, ")


# ---- full horizon at the BASELINE sizes (configs 3 and 4), into a second episode ---------
FULL_CASES = {
    "2perstage_lane": ("sc-2perstage-v0", 65536, {"kernel": "lane"}),
    "2perstage_nodes": ("sc-2perstage-v0", 65536, {"kernel": "nodes"}),
    "2perstage_stoch_nodes": ("sc-2perstage-v0", 65536, {"kernel": "nodes", "stochastic_leadtimes": True,
                                                          "avg_leadtime": 2, "max_leadtime": 4}),
    # two products: the auto kernel is the node-parallel one at one block per CU
    "2perstage_multiproduct": ("sc-2perstage-multiproduct-v0", 65536, {}),
    "ntom": ("sc-Nperstage-multiproduct-v0", 262144, dict(nodes_per_echelon=[8, 8, 8, 16])),
    "ntom_stoch": ("sc-Nperstage-multiproduct-v0", 262144,
                   dict(nodes_per_echelon=[8, 8, 8, 16], stochastic_leadtimes=True, avg_leadtime=2, max_leadtime=4)),
}


@pytest.mark.parametrize("case", sorted(FULL_CASES))
def test_full_horizon_episode_matches_oracle(case):
    """A whole 360-step episode at the BASELINE batch size, auto-reset into episode 2 and 3
    steps of it, with 32 sampled envs (block edges, first and last env included) compared
    with the oracle at every step: observations, rewards and done exactly, the terminal
    observation, the reset observation and the episode return. Heaps reach their peak
    occupancy over a full episode; check_errors() proves no in-transit heap overflowed."""
    import concurrent.futures as cf
    import multiprocessing as mp

    import gym_supplychain_amd as gsa
    from sc_replay import replay
    scenario, N, kw = FULL_CASES[case]
    kw = dict(kw)
    kernel = kw.pop("kernel", "auto")
    seed, extra = 1234, 3
    env = gsa.make_vec(scenario, N, seed=seed, device=DEV, obs_dtype=torch.float64, auto_reset=True, kernel=kernel,
                       **kw)
    sp = env.spec
    T = sp.total_time_steps
    sample = sorted({0, 1, 63, 64, 65, 127, 4095, 4096, N // 3, N // 2, N // 2 + 1, N - 65, N - 64, N - 2, N - 1} |
                    set(range(7, N, N // 17)))[:32]
    idx = torch.as_tensor(sample, device=DEV)
    obs0 = env.reset().index_select(0, idx).cpu().numpy()
    gen = torch.Generator(device=DEV).manual_seed(77)
    K = T + extra
    acts = np.zeros((K, len(sample), env.n_actions), dtype=np.float32)
    obs_rec = np.zeros((K, len(sample), env.n_obs))
    rew_rec = np.zeros((K, len(sample)))
    for k in range(K):
        a = torch.rand((N, env.n_actions), generator=gen, device=DEV, dtype=torch.float32) * 2.2 - 1.1
        obs, rew, done, info = env.step(a)
        acts[k] = a.index_select(0, idx).cpu().numpy()
        shown = info["terminal_observation"] if k == T - 1 else obs
        obs_rec[k] = shown.index_select(0, idx).cpu().numpy()
        rew_rec[k] = rew.index_select(0, idx).cpu().numpy()
        assert bool(done.all()) == (k == T - 1)
        if k == T - 1:
            reset_obs = obs.index_select(0, idx).cpu().numpy()
            final = info["episode_return"].index_select(0, idx).cpu().numpy()
    env.check_errors()
    nodes = gsa.envs.scenarios.SCENARIOS[scenario](**kw)[0]
    okw = dict(num_products=sp.P, demand_range=sp.demand_range, processing_ratio=sp.processing_ratio,
               stochastic_leadtimes=sp.stochastic_leadtimes, avg_leadtime=sp.avg_leadtime,
               max_leadtime=sp.max_leadtime, total_time_steps=T, **sp.penalties)
    jobs = [dict(env=n, nodes=nodes, okw=okw, seed=seed, R=sp.n_retailers, n_lt=sp.n_leadtimes,
                 lt=(sp.avg_leadtime, sp.max_leadtime), demand_range=sp.demand_range, acts=acts[:, j],
                 obs=obs_rec[:, j], rew=rew_rec[:, j], first_obs=obs0[j], reset_obs=reset_obs[j],
                 final_return=float(final[j]), T=T) for j, n in enumerate(sample)]
    with cf.ProcessPoolExecutor(max_workers=8, mp_context=mp.get_context("spawn")) as pool:
        results = list(pool.map(replay, jobs))
    bad = [(n, b) for n, b in results if b]
    assert not bad, bad[:3]


def test_lds_kernel_block_sizes_agree():
    """The LDS lane kernel runs 32 envs per block below two full waves per SIMD and 64 above
    (scg_supplychain.hip sc_lds_epb); an env's trajectory depends only on its global id, so
    the first envs of a small batch and of a large one must match bit for bit over a whole
    episode and into the next."""
    import gym_supplychain_amd as gsa
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    n_small, n_big = 1000, cus * 512 + 1000
    small = gsa.make_vec("sc-2perstage-v0", n_small, seed=5, device=DEV, obs_dtype=torch.float64, auto_reset=True,
                         kernel="lane")
    big = gsa.make_vec("sc-2perstage-v0", n_big, seed=5, device=DEV, obs_dtype=torch.float64, auto_reset=True,
                       kernel="lane")
    assert small.kernel_symbol.endswith(", 32>") and big.kernel_symbol.endswith(", 64>")
    o1, o2 = small.reset(), big.reset()
    assert torch.equal(o1, o2[:n_small])
    gen = torch.Generator(device=DEV).manual_seed(3)
    for t in range(small.spec.total_time_steps + 5):
        a = torch.rand((n_big, big.n_actions), generator=gen, device=DEV) * 2 - 1
        o1, r1, d1, _ = small.step(a[:n_small].contiguous())
        o2, r2, d2, _ = big.step(a)
        assert torch.equal(o1, o2[:n_small]) and torch.equal(r1, r2[:n_small]), t
    small.check_errors()
    big.check_errors()
