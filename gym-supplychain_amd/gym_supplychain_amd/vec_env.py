"""Stable-Baselines3-style VecEnv over the device batch envs.

The reference envs are single gym envs that an external trainer batches with SB3's
VecEnv (the `sc_` prefix of info['sc_episode'], supplychain_env.py:794-795,
exists for SB3's Monitor). Here the batch already lives on the GPU, so `SB3VecEnv`
presents a BeerGameVecEnv / BeerGame2VecEnv / SupplyChainVecEnv through SB3's VecEnv
contract instead of wrapping N Python envs:

    num_envs, observation_space / action_space (one env's spaces)
    reset() -> obs [N, ...]
    step_async(actions); step_wait() -> (obs, rewards float32 [N], dones bool [N], infos)
    auto-reset: the terminal step returns the next episode's first obs and
                infos[i]['terminal_observation']; with monitor=True also
                infos[i]['episode'] = {'r', 'l', 't'} (SB3 VecMonitor's keys)
    close(), seed(), get_attr/set_attr/env_method/env_is_wrapped, get_images()

Every env of a batch steps in lock-step, so all dones are equal. `numpy=True` (default,
what SB3 algorithms consume) copies obs/rewards to pinned host buffers once per step;
`numpy=False` returns the device tensors (views overwritten by the next step) for a
GPU-resident learner. When stable_baselines3 is importable the class subclasses its
VecEnv, so SB3 algorithms and wrappers accept it without DummyVecEnv; SB3 is not a
dependency.
"""
import time

import numpy as np
import torch

try:  # optional: SB3 is not part of this image
    from stable_baselines3.common.vec_env import VecEnv as _SB3VecEnv  # type: ignore
except ImportError:  # pragma: no cover - depends on the image
    _SB3VecEnv = object


class SB3VecEnv(_SB3VecEnv):
    """SB3 VecEnv view of a device batch env built with auto_reset=True."""

    def __init__(self, venv, numpy=True, monitor=True):
        if not getattr(venv, "auto_reset", False):
            raise ValueError("SB3VecEnv needs a batch env constructed with auto_reset=True")
        self.venv = venv
        if _SB3VecEnv is not object:
            super().__init__(int(venv.n_envs), venv.single_observation_space, venv.single_action_space)
        self.num_envs = int(venv.n_envs)
        self.observation_space = venv.single_observation_space
        self.action_space = venv.single_action_space
        self.render_mode = None
        self.numpy = bool(numpy)
        self.monitor = bool(monitor)
        self.horizon = int(venv.max_weeks) if hasattr(venv, "max_weeks") else int(venv.spec.total_time_steps)
        self._actions = None
        self._t0 = time.time()
        self._host = {}

    # ---------------------------------------------------------------- host copies
    def _to_host(self, name, t):
        """Copy a device tensor into a reused pinned buffer (one sync per step)."""
        buf = self._host.get(name)
        if buf is None or buf.shape != t.shape or buf.dtype != t.dtype:
            buf = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            self._host[name] = buf
        buf.copy_(t, non_blocking=True)
        return buf

    # ---------------------------------------------------------------- VecEnv API
    def reset(self):
        obs = self.venv.reset()
        if not self.numpy:
            return obs
        h = self._to_host("obs", obs)
        torch.cuda.current_stream(self.venv.device).synchronize()
        return h.numpy().copy()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        actions, self._actions = self._actions, None
        if actions is None:
            raise RuntimeError("step_wait() without step_async()")
        obs, rew, done, info = self.venv.step(actions)
        terminal = "terminal_observation" in info  # build_info puts 'sc_episode' in every info
        if not self.numpy:
            infos = self._infos(terminal, info, device=True)
            return obs, rew, done, infos
        h_obs = self._to_host("obs", obs)
        h_rew = self._to_host("rew", rew)
        if terminal:
            h_term = self._to_host("term", info["terminal_observation"])
            h_ret = self._to_host("ret", info["episode_return"]) if "episode_return" in info else None
        torch.cuda.current_stream(self.venv.device).synchronize()
        obs_np = h_obs.numpy().copy()
        rew_np = h_rew.numpy().astype(np.float32)
        dones = np.full(self.num_envs, terminal, dtype=bool)
        if not terminal:
            return obs_np, rew_np, dones, [{} for _ in range(self.num_envs)]
        term = h_term.numpy().copy()
        rets = h_ret.numpy().astype(np.float64) if h_ret is not None else None
        return obs_np, rew_np, dones, self._infos(True, None, term=term, rets=rets)

    def _infos(self, terminal, info, device=False, term=None, rets=None):
        if not terminal:
            return [{} for _ in range(self.num_envs)]
        if device:
            term = info["terminal_observation"]
            rets = info.get("episode_return")
            if rets is not None and self.monitor:  # one device->host copy, not one sync per env
                rets = rets.cpu().tolist()
        elapsed = round(time.time() - self._t0, 6)
        infos = []
        for i in range(self.num_envs):
            d = {"terminal_observation": term[i], "TimeLimit.truncated": False}
            if self.monitor and rets is not None:
                d["episode"] = {"r": float(rets[i]), "l": self.horizon, "t": elapsed}
            infos.append(d)
        return infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.venv.close()

    def seed(self, seed=None):
        """Re-key the batch's Philox streams; every env shares the key and differs by its
        global id, so one seed covers the batch (SB3 returns one entry per env)."""
        self.venv.seed(seed)
        return [seed] * self.num_envs

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def get_attr(self, attr_name, indices=None):
        value = getattr(self.venv, attr_name)
        idx = self._indices(indices)
        if isinstance(value, torch.Tensor) and value.dim() > 0 and value.shape[0] == self.num_envs:
            return [value[i] for i in idx]
        return [value for _ in idx]

    def set_attr(self, attr_name, value, indices=None):
        if indices is not None and len(list(self._indices(indices))) != self.num_envs:
            raise ValueError("attributes are batch-wide: set_attr applies to every env")
        setattr(self.venv, attr_name, value)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        result = getattr(self.venv, method_name)(*method_args, **method_kwargs)
        return [result for _ in self._indices(indices)]

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    def get_images(self):
        return [None for _ in range(self.num_envs)]

    def render(self, mode=None):
        return None
