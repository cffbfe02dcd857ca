"""Env classes, exported under the reference's names (gym_supplychain/envs/__init__.py:1-10)."""
from .beergame_env import BeerGame2VecEnv, BeerGameConfig, BeerGameEnv, BeerGameEnv2, BeerGameVecEnv  # noqa: F401
from .scenarios import (SCENARIOS, SupplyChain2perStageEnv, SupplyChain2perStageSeasonalEnv,  # noqa: F401
                        SupplyChainMultiProduct, SupplyChainMultiProduct_DemConfigByProd,
                        SupplyChainMultiProduct_DemConfigByProd_IncCosts, SupplyChainMultiProduct_IncreasingCosts,
                        SupplyChainNPerStage)
from .supplychain_env import SupplyChainEnv, SupplyChainSpec, SupplyChainVecEnv  # noqa: F401
