"""gym_supplychain_amd — MI355X-native vectorised environments of caburu/gym-supplychain.

Drop-in for the reference's hot path: the gym ids it registers (gym_supplychain/
__init__.py:1-51) map to classes with the reference's names and gym API, whose step()
dynamics run as fused HIP kernels through the C ABI in include/scgpu.h.

    import gym_supplychain_amd as gsa
    env = gsa.make("beergame-v0")                       # one env, reference API
    venv = gsa.make_vec("beergame-v0", 65536, demand="poisson", seed=0)   # batched
"""
from . import _native  # noqa: F401  (fails loudly when libscgpu.so is missing)
from .envs import (SCENARIOS, BeerGame2VecEnv, BeerGameEnv, BeerGameEnv2, BeerGameVecEnv, SupplyChain2perStageEnv,
                   SupplyChain2perStageSeasonalEnv, SupplyChainEnv, SupplyChainMultiProduct,
                   SupplyChainMultiProduct_DemConfigByProd, SupplyChainMultiProduct_DemConfigByProd_IncCosts,
                   SupplyChainMultiProduct_IncreasingCosts, SupplyChainNPerStage, SupplyChainVecEnv)
from .vec_env import SB3VecEnv

__all__ = ["BeerGameEnv", "BeerGameVecEnv", "BeerGameEnv2", "BeerGame2VecEnv", "SupplyChainEnv", "SupplyChainVecEnv", "SupplyChain2perStageEnv",
           "SupplyChainNPerStage", "SupplyChainMultiProduct", "SupplyChainMultiProduct_IncreasingCosts",
           "SupplyChain2perStageSeasonalEnv", "SupplyChainMultiProduct_DemConfigByProd",
           "SupplyChainMultiProduct_DemConfigByProd_IncCosts",
           "SB3VecEnv", "ENV_IDS", "VEC_ENV_IDS", "make", "make_vec", "register_gym"]

# id -> entry point, as registered by the reference (gym_supplychain/__init__.py:3-51).
ENV_IDS = {
    "beergame-v0": "gym_supplychain_amd.envs:BeerGameEnv",
    "beergame-v2": "gym_supplychain_amd.envs:BeerGameEnv2",
    "supplychain-v0": "gym_supplychain_amd.envs:SupplyChainEnv",
    "sc-2perstage-v0": "gym_supplychain_amd.envs:SupplyChain2perStageEnv",
    "sc-2perstage-multiproduct-v0": "gym_supplychain_amd.envs:SupplyChainMultiProduct",
    "sc-Nperstage-multiproduct-v0": "gym_supplychain_amd.envs:SupplyChainNPerStage",
    "sc-2perstage-multiproduct-inccosts-v0": "gym_supplychain_amd.envs:SupplyChainMultiProduct_IncreasingCosts",
    "sc-2perstage-seasonal-v0": "gym_supplychain_amd.envs:SupplyChain2perStageSeasonalEnv",
    "sc-2perstage-multiproduct-v1": "gym_supplychain_amd.envs:SupplyChainMultiProduct_DemConfigByProd",
    "sc-2perstage-multiproduct-inccosts-v1": "gym_supplychain_amd.envs:SupplyChainMultiProduct_DemConfigByProd_IncCosts",
}
_VEC_KEYS = ("seed", "device", "env_offset", "auto_reset", "obs_dtype", "track_returns", "kernel", "demand_table",
             "leadtime_table")


def _sc_vec(builder):
    def make(n_envs, **kw):
        vec_kw = {k: kw.pop(k) for k in _VEC_KEYS if k in kw}
        nodes, env_kw = builder(**kw)
        seed = env_kw.pop("seed", None)
        vec_kw.setdefault("seed", seed if seed is not None else 0)
        return SupplyChainVecEnv(n_envs, nodes, **vec_kw, **env_kw)
    return make


VEC_ENV_IDS = {
    "beergame-v0": BeerGameVecEnv,
    "beergame-v2": BeerGame2VecEnv,
    "supplychain-v0": SupplyChainVecEnv,
    **{env_id: _sc_vec(b) for env_id, b in SCENARIOS.items()},
}


def _resolve(entry_point):
    mod, _, name = entry_point.partition(":")
    import importlib
    return getattr(importlib.import_module(mod), name)


def make(id, **kwargs):
    """Construct the single-env class registered under `id` (gym.make equivalent)."""
    if id not in ENV_IDS:
        raise KeyError(f"unknown env id {id!r}; available: {sorted(ENV_IDS)}")
    return _resolve(ENV_IDS[id])(**kwargs)


def make_vec(id, n_envs, **kwargs):
    """Construct the batched (N envs per GPU) class for `id`."""
    if id not in VEC_ENV_IDS:
        raise KeyError(f"no vectorised env for {id!r}; available: {sorted(VEC_ENV_IDS)}")
    return VEC_ENV_IDS[id](n_envs, **kwargs)


def register_gym():
    """Register the ids with gym/gymnasium when one is installed (no-op otherwise)."""
    for modname in ("gymnasium", "gym"):
        try:
            reg = __import__(modname + ".envs.registration", fromlist=["register"])
        except ImportError:
            continue
        for env_id, ep in ENV_IDS.items():
            try:
                reg.register(id=env_id, entry_point=ep)
            except Exception:  # already registered
                pass
        return True
    return False
