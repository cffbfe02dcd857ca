"""Inert stand-in for the `gym` package, used ONLY in the survey/build container to
import /root/reference for golden-vector generation (oracle/gen_golden.py).

gym is not installed in this image and cannot be fetched. The reference's hot-path
arithmetic does not touch gym: BeerGameEnv only subclasses gym.Env
(gym_supplychain/envs/beergame_env.py:6) and SupplyChainEnv only declares its
spaces with gym.spaces.Box (gym_supplychain/envs/supplychain_env.py:625-626).
This stub therefore provides shape holders and no-ops; nothing here is sampled or
computed. Golden vectors are driven with explicit actions, never Box.sample().
Never shipped, never imported by the product or on the GPU box.
"""
from . import error, spaces, utils  # noqa: F401
from .envs import registration  # noqa: F401


class Env:
    metadata = {}
    action_space = None
    observation_space = None

    def seed(self, seed=None):
        return [seed]

    def close(self):
        pass
