"""SmartNanogridEnv: the single-environment gym surface of the reference
(smart_nanogrid_gym/envs/smart_nanogrid_environment.py), backed by the batched GPU
implementation with num_envs = 1.

Same constructor keywords, same spaces, reset() -> (obs, {}), step(a) ->
(obs float32[obs_dim], reward float64, terminated, False, {}).
"""
import ctypes

import numpy as np
import torch

from ._native import check, lib
from .recorder import DayRecorder
from .vec_env import SmartNanogridVecEnv, _raw_stream

try:  # subclass gym(nasium).Env when available so wrappers / checkers accept it
    import gymnasium as _gym   # pragma: no cover - not in the image
except Exception:
    try:
        import gym as _gym     # pragma: no cover
    except Exception:
        _gym = None

_Base = _gym.Env if _gym is not None else object



class SmartNanogridEnv(_Base):
    metadata = {"render_modes": []}

    def __init__(self, price_model=0, number_of_chargers=8, pv_system_available_in_model=True,
                 battery_system_available_in_model=True, vehicle_to_everything=False,
                 enable_different_vehicle_battery_capacities=True, enable_requested_state_of_charge=False,
                 algorithm_used="", environment_mode="", time_interval="", charging_mode="",
                 vehicle_uncharged_penalty_mode="", *, seed=0, device=0, rng="reference", results_directory=None,
                 **extra):
        """results_directory: write the reference's per-day prediction_results / initial_values
        files there (smart_nanogrid_environment.py:239-309; DayRecorder); None = no files."""
        self._venv = SmartNanogridVecEnv(
            1, seed=seed, device=device, rng=rng, price_model=price_model, number_of_chargers=number_of_chargers,
            pv_system_available_in_model=pv_system_available_in_model,
            battery_system_available_in_model=battery_system_available_in_model,
            vehicle_to_everything=vehicle_to_everything,
            enable_different_vehicle_battery_capacities=enable_different_vehicle_battery_capacities,
            enable_requested_state_of_charge=enable_requested_state_of_charge, algorithm_used=algorithm_used,
            environment_mode=environment_mode, time_interval=time_interval, charging_mode=charging_mode,
            vehicle_uncharged_penalty_mode=vehicle_uncharged_penalty_mode, **extra)
        self.observation_space = self._venv.observation_space
        self.action_space = self._venv.action_space
        self.NUMBER_OF_CHARGERS = self._venv.settings.number_of_chargers
        self.TIME_INTERVAL = self._venv.settings.time_interval
        self.simulated_single_day = False
        self.timestep = None
        self.recorder = DayRecorder(self._venv, [0], results_directory) if results_directory is not None else None
        # step(): "host" = one sng_step_host call (the step kernel reads the actions from and writes its outputs
        # to mapped host memory: one dispatch and one wait); "torch" = the VecEnv's device buffers with torch
        # copies (round 5's path; a recorder or per-step diagnostics need it, as they read device arrays)
        self.step_path = "host"
        v = self._venv
        # the host path's arguments, made once (an ndarray's .ctypes.data costs ~2.5 us per call)
        self._act1 = np.zeros(v.act_dim, np.float32)
        self._obs1 = np.zeros(v.obs_dim, np.float32)
        self._rew1 = np.zeros(1, np.float64)
        self._done1 = np.zeros(1, np.uint8)
        self._flags1 = np.zeros(1, np.uint32)
        self._io_args = [ctypes.c_void_p(x.ctypes.data)
                         for x in (self._act1, self._obs1, self._rew1, self._done1, self._flags1)]
        self._info_ref = ctypes.byref(v._info)
        self._dev_index = v.device.index or 0

    def reset(self, generate_new_initial_values=True, algorithm_used="", environment_mode="", **kwargs):
        """smart_nanogrid_environment.py:311-351 (gym-0.26 `seed=`/`options=` are accepted and ignored,
        as the reference swallows them in **kwargs).  generate_new_initial_values=False replays the last
        generated day with Requested_SOC cleared and a new PV ratio, as the reference's load_initial_values
        does (charging_station.py:119-136; what solvers/evaluator.py:88-101 relies on)."""
        obs = self._venv.reset(generate_new_initial_values, algorithm_used, environment_mode,
                               **{k: v for k, v in kwargs.items() if k not in ("seed", "options")})
        self.simulated_single_day = False
        self.timestep = 0
        return obs[0], {}

    def step(self, actions):
        """smart_nanogrid_environment.py:140-188.  After the day ends call reset() (the reference would
        silently re-run the day on its mutated arrays; this raises instead)."""
        if self.simulated_single_day:
            raise RuntimeError("the simulated day is over: call reset()")
        v = self._venv
        if self.step_path == "host" and not v._recorders and not v.info_d:
            if getattr(actions, "shape", None) == self._act1.shape:
                self._act1[:] = actions
            else:
                a = np.asarray(actions, dtype=np.float32).reshape(-1)
                if a.size != v.act_dim:
                    raise ValueError(f"actions must have {v.act_dim} elements")
                self._act1[:] = a
            check(lib().sng_step_host(v._h, *self._io_args, self._info_ref, _raw_stream(self._dev_index)), v._h)
            if self._flags1[0]:
                v._raise_flags(v._read_and_clear_flags())
            terminated = bool(self._done1[0])
            self.timestep = 0 if terminated else self.timestep + 1
            self.simulated_single_day = terminated
            return self._obs1.copy(), np.float64(self._rew1[0]), terminated, False, {}
        v._act_h.numpy()[0] = np.asarray(actions, dtype=np.float32).reshape(-1)
        with torch.cuda.device(v.device):
            v.actions_d.copy_(v._act_h, non_blocking=True)
            v.step_tensors(v.actions_d)
            v._out_h.copy_(v._out_d, non_blocking=True)   # reward, obs, done, flag summary
            torch.cuda.current_stream(v.device).synchronize()
        flags = v._step_flags()
        if flags is not None:
            v._raise_flags(flags)
        terminated = bool(v._done_h.numpy()[0])
        self.timestep = 0 if terminated else self.timestep + 1
        self.simulated_single_day = terminated
        return v._obs_h.numpy()[0].copy(), np.float64(v._rew_h.numpy()[0]), terminated, False, {}

    @property
    def random_pv_shift_ratio(self):
        """The day's PV shift ratio (smart_nanogrid_environment.py:65, :181, :349)."""
        return float(self._venv.pv_ratio()[0])

    def render(self, mode="human"):
        pass

    def seed(self, seed=None):
        pass

    def close(self):
        self._venv.close()

    @property
    def unwrapped(self):
        return self
