"""MI355X-native batched SmartNanogridEnv (drop-in for smart_nanogrid_gym's step()/reset()).

    from smart_nanogrid_gym import SmartNanogridEnv, SmartNanogridVecEnv

`SmartNanogridEnv-v0` is registered with gym / gymnasium when one of them is installed,
with the reference's id and max_episode_steps (smart_nanogrid_gym/__init__.py:4-8).
"""
from .envs import SmartNanogridEnv
from .evaluation import (RuleBasedController, evaluate_model_for_single_episode, evaluate_models, generate_days,
                         predict_single_day)
from .recorder import DayRecorder
from .settings import EnvSettings, parse_time_interval
from .vec_env import EpisodeGraph, SmartNanogridVecEnv

__all__ = ["SmartNanogridEnv", "SmartNanogridVecEnv", "EpisodeGraph", "EnvSettings", "DayRecorder",
           "parse_time_interval", "RuleBasedController", "evaluate_model_for_single_episode", "predict_single_day",
           "evaluate_models", "generate_days"]


def _register():
    for modname in ("gymnasium", "gym"):
        try:
            mod = __import__(modname + ".envs.registration", fromlist=["register"])
        except Exception:
            continue
        try:
            mod.register(id="SmartNanogridEnv-v0", entry_point="smart_nanogrid_gym.envs:SmartNanogridEnv",
                         max_episode_steps=200)
        except Exception:
            pass


_register()
