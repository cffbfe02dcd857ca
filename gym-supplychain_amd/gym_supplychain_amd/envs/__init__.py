"""Env classes, exported under the reference's names (gym_supplychain/envs/__init__.py:1-10)."""
from .beergame_env import BeerGameConfig, BeerGameEnv, BeerGameVecEnv  # noqa: F401
