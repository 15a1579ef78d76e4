"""A stand-in for stable-baselines3 2.x's abstract `VecEnv` (SB3 is not installed in this image).

It restates the parts of `stable_baselines3/common/vec_env/base_vec_env.py` (SB3 2.x) a VecEnv subclass
relies on: the constructor's state (`num_envs`, spaces, `reset_infos`, `_seeds`, `_options`, the
`get_attr("render_modes")` probe), the abstract methods, and the concrete `step`, `seed` and
`set_options`.  `load_vec_env_with_sb3()` imports a private copy of smart_nanogrid_gym/vec_env.py with
this stand-in installed as `stable_baselines3.common.vec_env`, leaving the package's own module alone.
The SB3 runtime itself stays parity-unpinned.
"""
import abc
import importlib.util
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VEC_ENV_PY = os.path.join(ROOT, "smart-nanogrid-gym_amd", "smart_nanogrid_gym", "vec_env.py")


class VecEnv(abc.ABC):
    def __init__(self, num_envs, observation_space, action_space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space
        self.reset_infos = [{} for _ in range(num_envs)]
        self._seeds = [None for _ in range(num_envs)]
        self._options = [{} for _ in range(num_envs)]
        try:
            render_modes = self.get_attr("render_modes")[0]
        except AttributeError:
            render_modes = []
        self.metadata = {"render_modes": render_modes}

    @abc.abstractmethod
    def reset(self):
        ...

    @abc.abstractmethod
    def step_async(self, actions):
        ...

    @abc.abstractmethod
    def step_wait(self):
        ...

    @abc.abstractmethod
    def close(self):
        ...

    @abc.abstractmethod
    def get_attr(self, attr_name, indices=None):
        ...

    @abc.abstractmethod
    def set_attr(self, attr_name, value, indices=None):
        ...

    @abc.abstractmethod
    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        ...

    @abc.abstractmethod
    def env_is_wrapped(self, wrapper_class, indices=None):
        ...

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def seed(self, seed=None):
        if seed is None:
            seed = int(np.random.randint(0, np.iinfo(np.uint32).max, dtype=np.uint32))
        self._seeds = [seed + idx for idx in range(self.num_envs)]
        return self._seeds

    def set_options(self, options=None):
        if options is None:
            options = {}
        self._options = [dict(options) for _ in range(self.num_envs)] if isinstance(options, dict) else list(options)


def _stub_modules():
    sb3 = types.ModuleType("stable_baselines3")
    common = types.ModuleType("stable_baselines3.common")
    vec = types.ModuleType("stable_baselines3.common.vec_env")
    vec.VecEnv = VecEnv
    sb3.common = common
    common.vec_env = vec
    return {"stable_baselines3": sb3, "stable_baselines3.common": common, "stable_baselines3.common.vec_env": vec}


def load_vec_env_with_sb3():
    """vec_env.py imported as `smart_nanogrid_gym._vec_env_sb3` with the stand-in on sys.modules."""
    import smart_nanogrid_gym  # noqa: F401  (the parent package of the private copy)
    mods = _stub_modules()
    saved = {k: sys.modules.get(k) for k in mods}
    sys.modules.update(mods)
    try:
        spec = importlib.util.spec_from_file_location("smart_nanogrid_gym._vec_env_sb3", VEC_ENV_PY)
        module = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(module)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return module


# The ways SB3 2.x's own code reads a VecEnv's `infos` (restated from its published sources, SB3 is not
# installed): each takes (obs, rewards, dones, infos) as step_wait returns them and gives what SB3 keeps.
def vec_monitor_step(rewards, dones, infos, returns, lengths):
    """VecMonitor.step_wait: `new_infos = list(infos[:])`, a copied dict with an "episode" entry for each done
    env, the running returns and lengths reset there."""
    returns += rewards
    lengths += 1
    new_infos = list(infos[:])
    for i in range(len(dones)):
        if dones[i]:
            info = infos[i].copy()
            info["episode"] = {"r": float(returns[i]), "l": int(lengths[i]), "t": 0.0}
            returns[i] = 0.0
            lengths[i] = 0
            new_infos[i] = info
    return new_infos


def update_info_buffer(infos, dones, ep_info_buffer):
    """BaseAlgorithm._update_info_buffer: every env's info is read with .get()."""
    for idx, info in enumerate(infos):
        maybe_ep_info = info.get("episode")
        if maybe_ep_info is not None:
            ep_info_buffer.append(maybe_ep_info)
        assert info.get("is_success") is None


def timeout_bootstrap_envs(dones, infos):
    """OnPolicyAlgorithm.collect_rollouts: the done envs whose day was truncated (their terminal_observation is
    bootstrapped through the value net)."""
    return [idx for idx, done in enumerate(dones)
            if done and infos[idx].get("terminal_observation") is not None
            and infos[idx].get("TimeLimit.truncated", False)]


def store_transition_next_obs(new_obs, dones, infos):
    """OffPolicyAlgorithm._store_transition: the next observation of a done env is its terminal_observation."""
    next_obs = new_obs.copy()
    for i, done in enumerate(dones):
        if done and infos[i].get("terminal_observation") is not None:
            next_obs[i] = infos[i]["terminal_observation"]
    return next_obs


def replay_buffer_timeouts(infos):
    """ReplayBuffer.add(handle_timeout_termination=True)."""
    return np.array([info.get("TimeLimit.truncated", False) for info in infos])


def vec_normalize_terminal(dones, infos, scale):
    """VecNormalize.step_wait: the done envs' terminal_observation is replaced in place."""
    for idx, done in enumerate(dones):
        if not done:
            continue
        if "terminal_observation" in infos[idx]:
            infos[idx]["terminal_observation"] = infos[idx]["terminal_observation"] * scale
