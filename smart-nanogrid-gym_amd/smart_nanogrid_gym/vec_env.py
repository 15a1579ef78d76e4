"""Batched SmartNanogridEnv: num_envs independent copies of the reference environment
stepped by one fused HIP kernel per timestep (libsng.so).

`SmartNanogridVecEnv` is a stable-baselines3 VecEnv: it subclasses
`stable_baselines3.common.vec_env.VecEnv` when SB3 is importable (SB3's BaseAlgorithm._wrap_env
takes an env as batched only through `isinstance(env, VecEnv)`, and wraps anything else in a
DummyVecEnv as ONE env -- solvers/RL/ppo_train.py:89-92), and `object` otherwise, as envs.py does
for gym.Env.  It follows SB3 2.x's VecEnv contract (reset / step_async / step_wait / get_attr /
set_attr / env_method / env_is_wrapped / seed / set_options / close, `reset_infos`) with the
DummyVecEnv conventions: seeds and options given by seed() / set_options() apply at the next
reset(), automatic reset at the end of the day and the final observation in
infos[i]['terminal_observation'].  SB3 is not installed in this image, so the SB3 runtime itself is
parity-unpinned; tests/test_vecenv_sb3_cpu.py checks the hierarchy against a stand-in of SB3 2.x's
abstract VecEnv.  `reset_tensors` / `step_tensors` keep everything on the GPU for device-resident
RL loops.

Reference behaviour mirrored per env (smart_nanogrid_gym/envs/smart_nanogrid_environment.py):
  reset()  -> new day, t = 0, BESS state of charge carried over (:311-351)
  reset(generate_new_initial_values=False) -> the last generated day replayed (:347-357)
  step(a)  -> (obs float32, reward = -total cost float64, terminated, truncated=False, {}) (:140-188)
  errors   -> the reference's ValueErrors, raised after the step that hit them
"""
import collections.abc
import ctypes
import itertools
import operator
import time
import warnings

import numpy as np

from . import _native
from ._native import check, lib
from .settings import (BESS_ABOVE_ONE, NEGATIVE_DEMAND, WRONG_CHARGING_MODE, WRONG_PENALTY_MODE, EnvSettings)
from .spaces import make_spaces

try:
    import torch
except Exception:  # pragma: no cover
    torch = None

try:  # SB3 attaches a batched env only when it is an instance of its VecEnv
    from stable_baselines3.common.vec_env import VecEnv as _VecEnvBase   # pragma: no cover - not in the image
except Exception:
    _VecEnvBase = object

SLOTS = 25


def _empty_infos(n):
    """n distinct empty dicts (SB3's per-env infos): dict() mapped over a repeat runs in C, about a quarter
    faster than a list comprehension of {} at 65,536 envs."""
    return list(itertools.starmap(dict, itertools.repeat((), n)))


class StepInfos(collections.abc.Sequence):
    """SB3's per-env `infos` of one step, list-compatible and made on access.

    DummyVecEnv returns a list of num_envs fresh dicts: {} for a running env, and for an env whose day just
    ended {"terminal_observation": its last observation, "TimeLimit.truncated": False} (solvers/RL/ppo_train.py
    hands the env to SB3, whose rollout reads infos[i] of done envs).  At 65,536 envs building those dicts cost
    ~0.5 ms every step and, once a day, ~5.5 ms for the terminal ones (a numpy row view each;
    profiles/r05_sb3_path.log).  Here an env's dict is built the first time it is indexed (`infos[i]`, then
    cached, so writes through it persist, as VecNormalize's `infos[i]["terminal_observation"] = ...` needs);
    iterating, slicing, `list(infos)`, `infos.copy()` and comparison build the dicts they cover in bulk.
    Whatever is built holds exactly what DummyVecEnv's dict would, including the `v2x_breakpoint` entries of
    the reference's V2X breakpoint (central_management_system.py:160-165).  Pickling and deep copies give a
    plain list."""

    __slots__ = ("_n", "_terminal", "_done", "_v2x", "_made", "_all")

    def __init__(self, n, terminal_obs=None, done=None, v2x=()):
        self._n = int(n)
        self._terminal = terminal_obs        # [n, obs_dim] array holding the done envs' last observations
        self._done = done                    # bool [n]: the envs whose dict carries terminal_observation
        self._v2x = frozenset(int(i) for i in v2x)
        self._made = {}                      # index -> the dict handed out
        self._all = None                     # the whole list, once built

    def __len__(self):
        return self._n

    def _make(self, i):
        d = self._made.get(i)
        if d is None:
            d = {}
            if self._terminal is not None and self._done[i]:
                d["terminal_observation"] = self._terminal[i]
                d["TimeLimit.truncated"] = False
            if i in self._v2x:
                d["v2x_breakpoint"] = True
            self._made[i] = d
        return d

    def _build_all(self):
        """Every env's dict, as one list (the dicts already handed out keep their identity)."""
        if self._all is None:
            n = self._n
            if self._terminal is not None and self._done.all():
                out = [{"terminal_observation": o, "TimeLimit.truncated": False} for o in self._terminal]
            elif self._terminal is not None:
                out = _empty_infos(n)
                for i in np.nonzero(self._done)[0].tolist():
                    out[i].update(terminal_observation=self._terminal[i], **{"TimeLimit.truncated": False})
            else:
                out = _empty_infos(n)   # dict() over a repeat, in C (~8 ns a dict)
            for i in self._v2x:
                out[i]["v2x_breakpoint"] = True
            for i, d in self._made.items():
                out[i] = d
            self._all = out   # from now on every access reads this list
            self._made = None
        return self._all

    def __getitem__(self, i):
        if isinstance(i, slice):
            if self._all is not None:
                return self._all[i]
            r = range(*i.indices(self._n))
            return self._build_all()[i] if len(r) > 64 else [self._make(k) for k in r]
        i = operator.index(i)
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError("infos index out of range")
        return self._make(i) if self._all is None else self._all[i]

    def __iter__(self):
        return iter(self._build_all())

    def __reversed__(self):
        return reversed(self._build_all())

    def copy(self):
        return list(self._build_all())

    def __eq__(self, other):
        if isinstance(other, StepInfos):
            other = other._build_all()
        return isinstance(other, list) and self._build_all() == other

    __hash__ = None

    def __add__(self, other):
        return self._build_all() + list(other)

    def __reduce__(self):
        return (list, (self._build_all(),))

    def __repr__(self):
        return f"StepInfos({self._build_all()!r})"


def _host_copy(pinned):
    """A fresh numpy copy of a pinned host tensor (torch's CPU copy runs on the intra-op threads: ~5x numpy's
    single-threaded copy for a step's 7.6 MB of observations at 65,536 envs)."""
    out = np.empty(tuple(pinned.shape), dtype=pinned.numpy().dtype)
    torch.from_numpy(out).copy_(pinned)
    return out


_get_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None) if torch is not None else None


def _raw_stream(index):
    """torch's current stream on device `index` as a hipStream_t (int): the raw handle when torch exposes it
    (~0.3 us; torch.cuda.current_stream builds a Stream object, ~2 us), else through current_stream."""
    if _get_raw_stream is not None:
        return _get_raw_stream(index)
    return torch.cuda.current_stream(index).cuda_stream


def _stream_handle(device):
    return ctypes.c_void_p(_raw_stream(device.index or 0))


class SmartNanogridVecEnv(_VecEnvBase):
    """num_envs parallel SmartNanogridEnv-v0 environments on one GPU.

    Parameters (besides the reference's own keyword arguments):
      seed   -- env i behaves like the reference after `np.random.seed(seed + i); random.seed(seed + i)`
      device -- HIP device index
      rng    -- 'reference' (host MT19937 streams, reference-exact days) or 'device' (counter-based hash streams on the GPU)
      info   -- True: also fill the per-step diagnostics (grid power, BESS SoC, penalties ...)
      env_offset -- global index of env 0 when one env population is sharded over GPUs
                    (parallel.shard_envs); env i then behaves as global env env_offset + i
    """

    metadata = {"render_modes": []}
    render_mode = None
    render_modes = ()   # what SB3's VecEnv.__init__ reads through get_attr("render_modes")

    def __init__(self, num_envs=1, *, seed=0, device=0, rng="reference", info=False, env_offset=0, **env_kwargs):
        if torch is None or not torch.cuda.is_available():
            raise RuntimeError("SmartNanogridVecEnv needs a HIP device (torch.cuda unavailable)")
        self.settings = EnvSettings(**env_kwargs)
        self.num_envs = int(num_envs)
        self.observation_space, self.action_space = make_spaces(self.settings)
        self.device = torch.device("cuda", device)
        self.rng_mode = _native.RNG_DEVICE if rng == "device" else _native.RNG_REFERENCE
        self._seed = int(seed)
        if self._seed < 0 or (self.rng_mode == _native.RNG_REFERENCE
                              and self._seed + int(env_offset) + int(num_envs) > 2 ** 32):
            raise ValueError(f"seed {self._seed}: reference-RNG env i is seeded seed + env_offset + i, which must "
                             "stay in numpy's [0, 2**32)")
        cfg = self.settings.to_native()
        h = ctypes.c_void_p()
        check(lib().sng_create(ctypes.byref(cfg), device, self.num_envs, self._seed, ctypes.byref(h)))
        self._h = h
        self.env_offset = int(env_offset)
        if self.env_offset:
            check(lib().sng_set_env_offset(h, self.env_offset), h)
        dims = _native.SngDims()
        check(lib().sng_get_dims(h, ctypes.byref(dims)), h)
        self.obs_dim, self.act_dim, self.timesteps = dims.obs_dim, dims.act_dim, dims.timesteps
        self.step_lanes = dims.step_lanes_per_env
        self.slots = dims.slots
        E, O = self.num_envs, self.obs_dim
        dev = self.device
        self.actions_d = torch.zeros((E, self.act_dim), dtype=torch.float32, device=dev)
        # What the numpy (SB3) path brings back after every step, as one device block with one pinned host
        # mirror, so a step costs one device-to-host copy: reward f64 [E] | obs f32 [E][O] | done u8 [E] |
        # the flag summary words (SngInfo.flag_summary, 4 KiB), sections 256 B aligned.
        al = lambda x: (x + 255) // 256 * 256   # noqa: E731
        o_obs = al(E * 8)
        o_done = al(o_obs + E * O * 4)
        o_flag = al(o_done + E)
        W = _native.FLAG_SUMMARY_WORDS
        self._out_d = torch.zeros(o_flag + 4 * W, dtype=torch.uint8, device=dev)
        self._out_h = torch.zeros(o_flag + 4 * W, dtype=torch.uint8, pin_memory=True)

        def views(buf):
            return (buf[:E * 8].view(torch.float64), buf[o_obs:o_obs + E * O * 4].view(torch.float32).view(E, O),
                    buf[o_done:o_done + E], buf[o_flag:o_flag + 4 * W].view(torch.int32))
        self.reward_d, self.obs_d, self.done_d, self.flag_summary_d = views(self._out_d)
        self._rew_h, self._obs_h, self._done_h, self._flag_summary_h = views(self._out_h)
        self.flags_d = torch.zeros(E, dtype=torch.int32, device=dev)   # per-step flags, with info=True
        self.return_d = torch.zeros(E, dtype=torch.float64, device=dev)
        self.info_d = {}
        self.charger_power_d = self.vehicle_soc_d = None
        self._recorders = []
        self._info = _native.SngInfo()
        # errors are watched through the summary word (touched only when an env raises a flag), so the
        # step stores no per-env flags; info=True adds the per-step per-env flags to the diagnostics
        self._info.flag_summary = self.flag_summary_d.data_ptr()
        self._info.episode_return = self.return_d.data_ptr()
        if info:
            self._enable_info()
        # pinned host mirror of the actions for the numpy (SB3) path
        self._act_h = torch.zeros((E, self.act_dim), dtype=torch.float32, pin_memory=True)
        # step_tensors' fixed arguments (the output buffers and SngInfo never move)
        self._dev_index = self.device.index or 0
        self._act_shape = torch.Size((E, self.act_dim))
        self._sng_step = lib().sng_step
        self._step_args = (ctypes.c_void_p(self.obs_d.data_ptr()), ctypes.c_void_p(self.reward_d.data_ptr()),
                           ctypes.c_void_p(self.done_d.data_ptr()), ctypes.byref(self._info))
        self._prof = None
        self._pending = None
        self._warned_breakpoint = False
        self._last_reset = None   # 'generated', 'replay' or 'injected': how the loaded day began
        self.closed = False
        # SB3 2.x VecEnv state: the reset infos (the reference's reset returns {}, :351), and the seeds /
        # options that seed() / set_options() leave for the next reset
        self.reset_infos = None
        self._seeds = [None] * E
        self._options = [{} for _ in range(E)]
        if _VecEnvBase is not object:   # pragma: no cover - SB3 is not in the image
            _VecEnvBase.__init__(self, E, self.observation_space, self.action_space)
            self.render_mode = None

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if not self.closed and getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            lib().sng_destroy(self._h)
            self._h = None
        self.closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _enable_info(self, per_charger=False):
        """Allocate the SngInfo diagnostics (and, per_charger, the [E, N] power / SoC arrays the
        day recorder reads); the step kernel writes them from then on."""
        E, N, dev = self.num_envs, self.settings.number_of_chargers, self.device
        if not self.info_d:
            self.info_d = {f: torch.zeros(E, dtype=torch.float64, device=dev) for f in _native.INFO_FIELDS}
            for f, t in self.info_d.items():
                setattr(self._info, f, t.data_ptr())
            self._info.flags = self.flags_d.data_ptr()
        if per_charger and self.charger_power_d is None:
            self.charger_power_d = torch.zeros((E, N), dtype=torch.float64, device=dev)
            self.vehicle_soc_d = torch.zeros((E, N), dtype=torch.float64, device=dev)
            self._info.charger_power = self.charger_power_d.data_ptr()
            self._info.vehicle_soc = self.vehicle_soc_d.data_ptr()

    def attach_recorder(self, recorder):
        """Called by DayRecorder: notified after every reset and step of this env batch."""
        self._enable_info(per_charger=True)
        self._recorders.append(recorder)

    def detach_recorder(self, recorder):
        self._recorders = [r for r in self._recorders if r is not recorder]

    @property
    def timestep(self):
        return lib().sng_get_timestep(self._h)

    def _check_mode(self):
        if self.settings.penalty_mode is None:   # charging_station.py:59-60 raises inside reset()
            raise ValueError(WRONG_PENALTY_MODE)

    # ------------------------------------------------------------------ device-resident API
    def reset_tensors(self, rng=None):
        """New day for every env; returns the t=0 observations (device tensor [E, obs_dim]).  A seed left by
        seed() takes effect here."""
        self._check_mode()
        self._apply_pending_seed()
        return self._new_day(rng)

    def _new_day(self, rng=None):
        mode = self.rng_mode if rng is None else (_native.RNG_DEVICE if rng == "device" else _native.RNG_REFERENCE)
        with torch.cuda.device(self.device):
            self.return_d.zero_()
            check(lib().sng_reset(self._h, mode, ctypes.c_void_p(self.obs_d.data_ptr()),
                                  _stream_handle(self.device)), self._h)
        self._last_reset = "generated"
        for r in self._recorders:
            r.day_started()
        return self.obs_d

    def replay_tensors(self):
        """reset(generate_new_initial_values=False) (smart_nanogrid_environment.py:347-357): every env replays
        the day it last generated, as the reference's load_initial_values (charging_station.py:119-136)
        re-reads the initial_values.json its generation wrote -- same vehicles, Requested_SOC cleared to 0
        (so no vehicle penalty), a new PV ratio from the env's stream, BESS carried over.  Returns the t=0
        observations (device tensor).  The reference's file is one per process; here each env replays its
        own last generated day."""
        self._check_mode()
        self._apply_pending_seed()
        with torch.cuda.device(self.device):
            self.return_d.zero_()
            check(lib().sng_reset_replay(self._h, ctypes.c_void_p(self.obs_d.data_ptr()),
                                         _stream_handle(self.device)), self._h)
        self._last_reset = "replay"
        for r in self._recorders:
            r.day_started()
        return self.obs_d

    def step_tensors(self, actions):
        """One step for every env from device actions [E, act_dim] float32.
        Returns (obs [E, obs_dim] f32, reward [E] f64, done [E] u8) device tensors, no auto-reset.
        The call only enqueues the step on torch's current stream of the env's device (sng_step selects the
        device itself); its fixed arguments are built once, so the host keeps ahead of a ~6 us step
        (profiles/r06_reset_bench.log: an eager day of step_tensors calls)."""
        if (actions.dtype != torch.float32 or actions.get_device() != self._dev_index
                or not actions.is_contiguous()):
            actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        if actions.shape != self._act_shape:
            raise ValueError(f"actions must have shape {(self.num_envs, self.act_dim)}")
        rc = self._sng_step(self._h, actions.data_ptr(), *self._step_args, _raw_stream(self._dev_index))
        if rc:
            check(rc, self._h)
        for r in self._recorders:
            r.step_done(actions)
        return self.obs_d, self.reward_d, self.done_d

    def step_kernel_name(self):
        """The step kernel the next step_tensors launches, as rocprofv3 names it (sng_step_kernel_name)."""
        buf = ctypes.create_string_buffer(128)
        check(lib().sng_step_kernel_name(self._h, ctypes.byref(self._info), buf, len(buf)), self._h)
        return buf.value.decode()

    def reset_from_initial_values(self, initial_values, pv_ratio=None, restore_requested_soc=False):
        """Start a day from the reference's initial_values.json dicts (charging_station.py:164-180): one
        dict (broadcast to all envs) or a list of num_envs dicts.  The reference's load_initial_values
        (charging_station.py:119-136) does not restore 'Requested_SOC' (left at 0);
        restore_requested_soc=True uses the recorded values instead.  pv_ratio None: each env draws its
        ratio from its Python stream (smart_nanogrid_environment.py:349), as a reset does.
        """
        self._check_mode()
        E, N = self.num_envs, self.settings.number_of_chargers
        items = initial_values if isinstance(initial_values, (list, tuple)) else [initial_values] * E
        if len(items) != E:
            raise ValueError("need one initial_values dict per env")
        V = max(1, max(len(a) for d in items for a in d["Arrivals"]))
        S = self.slots
        soc = np.zeros((E, N, S))
        occ = np.zeros((E, N, S))
        cap = np.zeros((E, N, S))
        req = np.zeros((E, N, S))
        arr = np.full((E, N, V), -1, np.int32)
        dep = np.full((E, N, V), -1, np.int32)
        for i, d in enumerate(items):
            soc[i] = np.asarray(d["SOC"], np.float64)
            occ[i] = np.asarray(d["Charger_occupancy"], np.float64)
            cap[i] = np.asarray(d["Vehicle_capacities"], np.float64)
            if restore_requested_soc and "Requested_SOC" in d:
                req[i] = np.asarray(d["Requested_SOC"], np.float64)
            for c in range(N):
                arr[i, c, :len(d["Arrivals"][c])] = d["Arrivals"][c]
                dep[i, c, :len(d["Departures"][c])] = d["Departures"][c]
        ratio = None if pv_ratio is None else np.broadcast_to(np.asarray(pv_ratio, np.float64), (E,)).copy()
        return self.reset_from_arrays(soc, occ, cap, req, arr, dep, ratio)

    def reset_from_arrays(self, soc, occupancy, capacity, requested_soc, arrivals, departures, pv_ratio=None):
        """Start a day from explicit reference-layout arrays ([E, N, slots] / [E, N, V], -1 padded;
        slots = 25, or T+1 with the build-defined extended day).  pv_ratio None: drawn per env from its
        Python stream."""
        self._check_mode()
        seed = self._seed if self._seeds[0] is None else self._seeds[0]   # a pending seed() or the current one
        if pv_ratio is None and seed is not None:   # (after load_state the blob's seed: the library checks it)
            self._check_python_stream_seed(seed)
        self._apply_pending_seed()
        arrs = [np.ascontiguousarray(a, np.float64) for a in (soc, occupancy, capacity, requested_soc)]
        ai = np.ascontiguousarray(arrivals, np.int32)
        di = np.ascontiguousarray(departures, np.int32)
        sc = _native.SngScenario()
        if arrs[0].shape[-1] != self.slots:
            raise ValueError(f"scenario arrays need {self.slots} slots per charger")
        sc.slots = self.slots
        sc.max_vehicles = ai.shape[-1]
        sc.soc, sc.occupancy, sc.capacity, sc.requested_soc = [a.ctypes.data_as(_native.c_double_p) for a in arrs]
        sc.arrivals = ai.ctypes.data_as(_native.c_int32_p)
        sc.departures = di.ctypes.data_as(_native.c_int32_p)
        if pv_ratio is not None:
            ratio = np.ascontiguousarray(np.broadcast_to(np.asarray(pv_ratio, np.float64), (self.num_envs,)))
            sc.pv_ratio = ratio.ctypes.data_as(_native.c_double_p)
        with torch.cuda.device(self.device):
            self.return_d.zero_()
            check(lib().sng_reset_from_scenario(self._h, ctypes.byref(sc), ctypes.c_void_p(self.obs_d.data_ptr()),
                                                _stream_handle(self.device)), self._h)
            torch.cuda.current_stream(self.device).synchronize()
        self._last_reset = "injected"
        for r in self._recorders:
            r.day_started()
        return self._obs_to_host()

    # ------------------------------------------------------------------ SB3 VecEnv API
    _RESET_OPTIONS = ("generate_new_initial_values", "algorithm_used", "environment_mode", "initial_values",
                      "pv_ratio", "restore_requested_soc")

    def reset(self, generate_new_initial_values=True, algorithm_used="", environment_mode="", **kwargs):
        """smart_nanogrid_environment.py:311-351.  generate_new_initial_values=False replays the last
        generated day (replay_tensors); with initial_values=<dict or list> (and optionally pv_ratio=,
        restore_requested_soc=) it starts from those days instead (reset_from_initial_values).

        SB3 2.x: the seeds of seed() and the options of set_options() apply here, then are cleared
        (DummyVecEnv.reset).  The options are this method's keyword arguments; every env of the batch
        resets alike, so per-env options must all be equal."""
        opts = self._options
        self._options = [{} for _ in range(self.num_envs)]
        if any(opts):
            if any(o != opts[0] for o in opts):
                raise ValueError("set_options: every env of the batch resets alike; give one options dict")
            unknown = set(opts[0]) - set(self._RESET_OPTIONS)
            if unknown:
                raise ValueError(f"set_options: unknown reset options {sorted(unknown)}")
            o = dict(opts[0])
            generate_new_initial_values = o.pop("generate_new_initial_values", generate_new_initial_values)
            algorithm_used = o.pop("algorithm_used", algorithm_used)
            environment_mode = o.pop("environment_mode", environment_mode)
            kwargs = {**o, **kwargs}
        self.reset_infos = None   # the reference's reset returns {} per env (:351): made on first access
        if algorithm_used:
            self.settings.algorithm_used = algorithm_used
        if environment_mode:
            self.settings.environment_mode = environment_mode
        if not generate_new_initial_values:
            if "initial_values" in kwargs:
                return self.reset_from_initial_values(kwargs["initial_values"], kwargs.get("pv_ratio"),
                                                      kwargs.get("restore_requested_soc", False))
            self.replay_tensors()
            return self._obs_to_host()
        self.reset_tensors()
        return self._obs_to_host()

    def step_async(self, actions):
        self._pending = actions

    def step_wait(self):
        """The numpy step SB3 drives (DummyVecEnv semantics).  Device work: the actions' H2D copy, the step and
        one D2H copy of its outputs (reward, observation, done, flag summary).  A done step (the day's last)
        raises the day's flags, then enqueues the automatic reset (the next day and its observation's D2H
        copy), and the host copies the terminal observations while the device resets.  The infos are a
        StepInfos: each env's dict (terminal_observation on a done step) is made when it is first accessed.
        Host copies of the observations go through torch's multi-threaded CPU copy (a fresh array per step,
        as DummyVecEnv returns copies)."""
        actions = self._pending
        self._pending = None
        E = self.num_envs
        prof = self._prof
        t0 = time.perf_counter() if prof is not None else 0.0
        a = np.asarray(actions, dtype=np.float32).reshape(E, self.act_dim)
        self._act_h.copy_(torch.from_numpy(a))
        if prof is not None:
            ta = time.perf_counter()
        stream = torch.cuda.current_stream(self.device)
        with torch.cuda.device(self.device):
            if prof is not None:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
                ev[0].record(stream)
            self.actions_d.copy_(self._act_h, non_blocking=True)
            if prof is not None:
                ev[1].record(stream)
            self.step_tensors(self.actions_d)
            if prof is not None:
                ev[2].record(stream)
            self._out_h.copy_(self._out_d, non_blocking=True)   # reward, obs, done, flag summary: one copy
            if prof is not None:
                ev[3].record(stream)
                t1 = time.perf_counter()
            stream.synchronize()
        if prof is not None:
            t2 = time.perf_counter()
        flags = self._step_flags()
        if flags is not None:
            self._raise_flags(flags)
        obs = _host_copy(self._obs_h)
        rewards = _host_copy(self._rew_h)
        dones = self._done_h.numpy().astype(bool)
        v2x = () if flags is None else np.nonzero(flags & _native.FLAG_V2X_BREAKPOINT)[0].tolist()
        if prof is not None:
            t3 = time.perf_counter()
        if dones.any():
            # DummyVecEnv's automatic reset: a new day (seeds and options left by seed() / set_options() wait
            # for the caller's next reset()), enqueued before the terminal infos are built on the host
            self._check_mode()
            with torch.cuda.device(self.device):
                if prof is not None:
                    ev[4].record(stream)
                self._new_day()
                self._obs_h.copy_(self.obs_d, non_blocking=True)
                if prof is not None:
                    ev[5].record(stream)
                    t4 = time.perf_counter()
                # the terminal observations stay in `obs` (this step's fresh copy); each env's
                # terminal_observation is a row of it, made when its info is accessed
                infos = StepInfos(E, obs, dones, v2x)
                if prof is not None:
                    t5 = time.perf_counter()
                stream.synchronize()
            self.reset_infos = None   # made on first access
            if prof is not None:
                t6 = time.perf_counter()
            obs = _host_copy(self._obs_h)
            if prof is not None:
                t7 = time.perf_counter()
                for k, x in (("reset_enqueue", t4 - t3), ("terminal_infos", t5 - t4), ("reset_wait", t6 - t5),
                             ("reset_copy", t7 - t6), ("reset", t7 - t3)):
                    prof.setdefault(k, []).append(x)
                prof.setdefault("reset_device", []).append(ev[4].elapsed_time(ev[5]) * 1e-3)
        else:
            infos = StepInfos(E, v2x=v2x)
        if prof is not None:
            for k, x in (("actions_in", ta - t0), ("enqueue", t1 - ta), ("sync", t2 - t1), ("host_out", t3 - t2)):
                prof.setdefault(k, []).append(x)
            for k, (x, y) in (("h2d", (0, 1)), ("step", (1, 2)), ("d2h", (2, 3))):
                prof.setdefault(k, []).append(ev[x].elapsed_time(ev[y]) * 1e-3)
        return obs, rewards, dones, infos

    def _step_flags(self):
        """After a step's outputs reached the host: None when no env raised a flag since the last check
        (the summary word, copied with the outputs, is 0), else the per-env SNG_FLAG_* raised since then
        (the sticky flags, read and cleared; the summary is zeroed)."""
        if not self._flag_summary_h.numpy().any():
            return None
        return self._read_and_clear_flags()

    def _read_and_clear_flags(self):
        flags = np.zeros(self.num_envs, np.uint32)
        with torch.cuda.device(self.device):
            self.flag_summary_d.zero_()
            check(lib().sng_read_errors(self._h, flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 1,
                                        _stream_handle(self.device)), self._h)
        self._flag_summary_h.zero_()
        return flags.view(np.int32)

    def check_errors(self):
        """Raise the reference's exception for any flag an env raised since the last check (the device
        path, step_tensors, raises nothing by itself); synchronises the current stream."""
        with torch.cuda.device(self.device):
            self._flag_summary_h.copy_(self.flag_summary_d)
        flags = self._step_flags()
        if flags is not None:
            self._raise_flags(flags)

    def profile_phases(self, on=True):
        """Time the phases of every numpy step() (tools/sb3_path_bench.py): on=True starts recording,
        on=False stops and returns {phase: [seconds per step]}."""
        out = self._prof
        self._prof = {} if on else None
        return out

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def seed(self, seed=None):
        """SB3 2.x VecEnv.seed: env i draws the streams of seed + i from the next reset on (reference RNG: what
        np.random.seed(seed + i); random.seed(seed + i) gives the reference; device RNG: the hash streams of
        that seed from its first day).  seed=None picks a fresh seed.  Returns the per-env seeds.  The
        reference's own seed() is a no-op (smart_nanogrid_environment.py:362-365) and it seeds through the
        global RNGs instead."""
        top = 2 ** 32 - self.num_envs - self.env_offset   # np.random.seed takes [0, 2^32): seed + offset + i too
        if seed is None:
            seed = int(np.random.randint(0, max(top, 0) + 1, dtype=np.int64))
        seed = int(seed)
        if seed < 0 or (self.rng_mode == _native.RNG_REFERENCE and seed > top):
            raise ValueError(f"seed {seed}: reference-RNG env i is seeded seed + env_offset + i, which must stay "
                             f"in numpy's [0, 2**32); use a seed in [0, {top}]")
        self._seeds = [seed + i for i in range(self.num_envs)]
        return list(self._seeds)

    def set_options(self, options=None):
        """SB3 2.x VecEnv.set_options: keyword arguments of the next reset() (one dict for every env, or a
        list of num_envs equal dicts)."""
        if options is None:
            options = {}
        opts = ([dict(options) for _ in range(self.num_envs)] if isinstance(options, dict)
                else [dict(o) for o in options])
        if len(opts) != self.num_envs:
            raise ValueError("set_options: need one options dict per env")
        self._options = opts

    def _check_python_stream_seed(self, seed):
        """a day injected without pv_ratio draws each env's ratio from its Python stream,
        random.seed(seed + env_offset + i), in every RNG mode; the streams are seeded as numpy's are, so the
        last env's seed must stay below 2^32 here too (a device-RNG env accepts larger seeds otherwise)."""
        if seed + self.env_offset + self.num_envs > 2 ** 32:
            raise ValueError(f"seed {seed}: a day injected without pv_ratio draws env i's PV ratio from the Python "
                             f"stream random.seed(seed + env_offset + i), which must stay below 2**32; pass pv_ratio "
                             f"or use a seed in [0, {2 ** 32 - self.env_offset - self.num_envs}]")

    def _apply_pending_seed(self):
        if self._seeds[0] is None:
            return
        seed = self._seeds[0]
        with torch.cuda.device(self.device):
            check(lib().sng_set_seed(self._h, seed, _stream_handle(self.device)), self._h)
        self._seed = seed
        self._seeds = [None] * self.num_envs

    def render(self, mode="human"):
        return None

    @property
    def reset_infos(self):
        """SB3 2.x: the info dict of every env's last reset ({} per env, as the reference's reset returns)."""
        if self._reset_infos is None:
            self._reset_infos = [{} for _ in range(self.num_envs)]
        return self._reset_infos

    @reset_infos.setter
    def reset_infos(self, value):
        self._reset_infos = value

    # Per-env attributes get_attr / set_attr resolve env by env (the rest are shared by the batch: the
    # reference's constructor keywords, settings, spaces, the timestep).
    _PER_ENV_GET = {"random_pv_shift_ratio": "pv_ratio", "battery_state_of_charge": "battery_state_of_charge",
                    "vehicle_state_of_charge": "vehicle_state_of_charge"}
    _PER_ENV_SET = {"battery_state_of_charge": ("battery_state_of_charge", "set_battery_state_of_charge"),
                    "vehicle_state_of_charge": ("vehicle_state_of_charge", "set_vehicle_state_of_charge")}

    def get_attr(self, attr_name, indices=None):
        """SB3 VecEnv.get_attr: the attribute's value for each env of `indices` (AttributeError if unknown)."""
        idx = self._idx(indices)
        if attr_name in self._PER_ENV_GET:
            values = getattr(self, self._PER_ENV_GET[attr_name])()
            return [values[i] for i in idx]
        if attr_name in ("timestep",):
            return [self.timestep for _ in idx]
        for owner in (self.settings, self):
            if hasattr(owner, attr_name):
                v = getattr(owner, attr_name)
                return [v for _ in idx]
        raise AttributeError(f"SmartNanogridVecEnv has no attribute {attr_name!r}")

    def set_attr(self, attr_name, value, indices=None):
        """SB3 VecEnv.set_attr.  Per-env state (battery / vehicle state of charge) is set for the given envs
        only; a batch-wide setting (the constructor keywords, settings) can only be set for every env."""
        idx = self._idx(indices)
        if attr_name in self._PER_ENV_SET:
            getter, setter = self._PER_ENV_SET[attr_name]
            cur = getattr(self, getter)()
            cur[idx] = value
            getattr(self, setter)(cur)
            return
        if sorted(set(idx)) != list(range(self.num_envs)):
            raise ValueError(f"{attr_name!r} is shared by every env of the batch: set it with indices=None")
        if hasattr(self.settings, attr_name):
            setattr(self.settings, attr_name, value)
        elif hasattr(self, attr_name):
            setattr(self, attr_name, value)
        else:
            raise AttributeError(f"SmartNanogridVecEnv has no attribute {attr_name!r}")

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        """SB3 VecEnv.env_method: one result per env of `indices`.  get_scenario is called per env; a
        method that returns per-env values (an array with num_envs rows) is sliced per env; any other
        method acts on the whole batch and needs indices=None."""
        idx = self._idx(indices)
        if method_name == "get_scenario":
            return [self.get_scenario(i, *method_args, **method_kwargs) for i in idx]
        fn = getattr(self, method_name)
        if method_name not in self._PER_ENV_QUERIES and sorted(set(idx)) != list(range(self.num_envs)):
            raise ValueError(f"{method_name!r} acts on the whole batch: call it with indices=None")
        out = fn(*method_args, **method_kwargs)
        if isinstance(out, (np.ndarray, list, tuple)) and len(out) == self.num_envs:
            return [out[i] for i in idx]
        return [out for _ in idx]

    _PER_ENV_QUERIES = {"battery_state_of_charge", "pv_ratio", "vehicle_state_of_charge", "last_info_rows"}

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._idx(indices)]

    def get_images(self):
        return []

    def _idx(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, (int, np.integer)):
            indices = [int(indices)]
        idx = [int(i) for i in indices]
        if any(i < 0 or i >= self.num_envs for i in idx):
            raise IndexError("env index out of range")
        return idx

    # ------------------------------------------------------------------ helpers
    def _obs_to_host(self):
        self._obs_h.copy_(self.obs_d, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return _host_copy(self._obs_h)

    def _raise_flags(self, flags):
        if not flags.any():
            return
        f = int(np.bitwise_or.reduce(flags))
        if f & _native.FLAG_NEGATIVE_DEMAND:
            raise ValueError(NEGATIVE_DEMAND)
        if f & _native.FLAG_CHARGING_MODE:
            raise ValueError(WRONG_CHARGING_MODE)
        if f & _native.FLAG_BESS_SOC_ABOVE_1:
            raise ValueError(BESS_ABOVE_ONE)
        if f & _native.FLAG_V2X_BREAKPOINT and not self._warned_breakpoint:
            self._warned_breakpoint = True
            warnings.warn("V2X total power demand < 0: the reference stops in breakpoint() here "
                          "(central_management_system.py:160-165); continuing", RuntimeWarning)

    def last_info(self):
        """Per-step diagnostics of the last step (numpy, names of the reference results dict)."""
        torch.cuda.current_stream(self.device).synchronize()
        out = {k: v.cpu().numpy() for k, v in self.info_d.items()}
        if self.info_d:   # the last step's per-env flags (written with the diagnostics)
            out["flags"] = self.flags_d.cpu().numpy()
        else:             # the sticky flags raised since the last check (not cleared here)
            flags = np.zeros(self.num_envs, np.uint32)
            check(lib().sng_read_errors(self._h, flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 0,
                                        _stream_handle(self.device)), self._h)
            out["flags"] = flags.view(np.int32)
        out["episode_return"] = self.return_d.cpu().numpy()
        return out

    def last_info_rows(self):
        """last_info() as one dict per env."""
        info = self.last_info()
        return [{k: v[i] for k, v in info.items()} for i in range(self.num_envs)]

    def _host_array(self, fn, shape, value=None):
        out = np.zeros(shape) if value is None else np.ascontiguousarray(np.broadcast_to(
            np.asarray(value, np.float64), shape))
        with torch.cuda.device(self.device):
            check(fn(self._h, out.ctypes.data_as(_native.c_double_p), _stream_handle(self.device)), self._h)
        return out

    def battery_state_of_charge(self):
        return self._host_array(lib().sng_get_battery_soc, (self.num_envs,))

    def set_battery_state_of_charge(self, soc):
        self._host_array(lib().sng_set_battery_soc, (self.num_envs,), soc)

    def pv_ratio(self):
        return self._host_array(lib().sng_get_pv_ratio, (self.num_envs,))

    def vehicle_state_of_charge(self):
        return self._host_array(lib().sng_get_vehicle_soc, (self.num_envs, self.settings.number_of_chargers))

    def set_vehicle_state_of_charge(self, soc):
        self._host_array(lib().sng_set_vehicle_soc, (self.num_envs, self.settings.number_of_chargers), soc)

    def day_counter(self):
        """Device-RNG days started so far (the day the next device reset draws)."""
        out = ctypes.c_uint64()
        with torch.cuda.device(self.device):
            check(lib().sng_get_day_counter(self._h, ctypes.byref(out), _stream_handle(self.device)), self._h)
        return out.value

    # ------------------------------------------------------------------ checkpoint / resume
    def save_state(self):
        """The whole simulation state (sng_get_state: EV and BESS SoC, the loaded day, timestep, day counter,
        RNG streams, the running day returns) as bytes, for load_state on a handle of the same configuration."""
        size = ctypes.c_size_t()
        check(lib().sng_state_size(self._h, 1, ctypes.byref(size)), self._h)
        buf = np.empty(size.value, np.uint8)
        with torch.cuda.device(self.device):
            check(lib().sng_get_state(self._h, buf.ctypes.data_as(ctypes.c_void_p), size.value,
                                      ctypes.c_void_p(self.return_d.data_ptr()), _stream_handle(self.device)),
                  self._h)
        return buf.tobytes()

    def load_state(self, blob):
        """Restore a save_state() blob (the day continues from its timestep)."""
        buf = np.frombuffer(blob, np.uint8)
        with torch.cuda.device(self.device):
            check(lib().sng_set_state(self._h, buf.ctypes.data_as(ctypes.c_void_p), buf.size,
                                      ctypes.c_void_p(self.return_d.data_ptr()), _stream_handle(self.device)),
                  self._h)
        self._seed = None
        # the blob carries its own seed and streams: a seed() or set_options() left for the next reset
        # before the restore would re-seed the restored streams and reset the day counter there
        self._seeds = [None] * self.num_envs
        self._options = [{} for _ in range(self.num_envs)]
        # the blob's sticky per-env flags replace the handle's, so the summary word is rebuilt from
        # them: a stale summary would report flags the restored day never raised, and restored flags that were
        # never reported are raised (or reported as v2x_breakpoint infos) at the next step, as after any step
        flags = np.zeros(self.num_envs, np.uint32)
        with torch.cuda.device(self.device):
            check(lib().sng_read_errors(self._h, flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 0,
                                        _stream_handle(self.device)), self._h)
            self.flag_summary_d.zero_()
            self.flag_summary_d[0] = int(np.bitwise_or.reduce(flags)) if flags.size else 0
        self._flag_summary_h.zero_()

    # ------------------------------------------------------------------ the loaded day
    def get_scenarios(self, first=0, count=None, max_vehicles=8):
        """The current days of envs [first, first + count) as the reference's initial_values.json dicts
        (ChargingStation.generated_initial_values_json, charging_station.py:164-191) and their PV ratios,
        decoded from the device timeline (sng_get_scenario in include/sng.h)."""
        count = self.num_envs - first if count is None else int(count)
        N, S, V = self.settings.number_of_chargers, self.slots, int(max_vehicles)
        f = [np.zeros((count, N, S)) for _ in range(4)]
        arr = np.full((count, N, V), -1, np.int32)
        dep = np.full((count, N, V), -1, np.int32)
        nv = np.zeros((count, N), np.int32)
        ratio = np.zeros(count)
        P, I = _native.c_double_p, _native.c_int32_p
        with torch.cuda.device(self.device):
            check(lib().sng_get_scenario(self._h, int(first), count, V, *[a.ctypes.data_as(P) for a in f],
                                         arr.ctypes.data_as(I), dep.ctypes.data_as(I), nv.ctypes.data_as(I),
                                         ratio.ctypes.data_as(P), _stream_handle(self.device)), self._h)
        if (nv > V).any():
            return self.get_scenarios(first, count, int(nv.max()))
        soc, occ, cap, req = f
        out = []
        for k in range(count):
            out.append({"SOC": soc[k].tolist(), "Arrivals": [arr[k, c, :nv[k, c]].tolist() for c in range(N)],
                        "Departures": [dep[k, c, :nv[k, c]].tolist() for c in range(N)],
                        "Charger_occupancy": occ[k].tolist(), "Vehicle_capacities": cap[k].tolist(),
                        "Requested_SOC": req[k].tolist()})
        return out, ratio

    def get_scenario(self, env_index=0, max_vehicles=8):
        """The current day of env `env_index` (get_scenarios for one env): (initial_values dict, PV ratio)."""
        ivs, ratio = self.get_scenarios(int(env_index), 1, max_vehicles)
        return ivs[0], float(ratio[0])

    def run_eager_days(self, actions, days=1):
        """`days` device-RNG days (reset + T steps each) launched eagerly from C, back to back, without
        per-dispatch events (sng_time_step_kernels with ms = NULL); synchronises.  A seed left by seed()
        takes effect here (these days begin with resets)."""
        self._apply_pending_seed()
        a = actions.contiguous()
        with torch.cuda.device(self.device):
            check(lib().sng_time_step_kernels(self._h, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(self.obs_d.data_ptr()),
                                              ctypes.c_void_p(self.reward_d.data_ptr()),
                                              ctypes.c_void_p(self.done_d.data_ptr()), ctypes.byref(self._info),
                                              days, None, None, _stream_handle(self.device)), self._h)

    def time_step_kernels(self, actions, days=1, with_resets=False):
        """Device time (ms) of every step kernel over `days` eager device-RNG days, from HIP
        start/stop events attached to each kernel dispatch; actions [T, E, act_dim] on the device.
        with_resets: also return every day's reset time (ms), as (steps, resets).  A seed left by seed() takes
        effect here (these days begin with resets)."""
        self._apply_pending_seed()
        a = actions.contiguous()
        out = np.zeros(days * self.timesteps, np.float32)
        res = np.zeros(days, np.float32) if with_resets else None
        with torch.cuda.device(self.device):
            check(lib().sng_time_step_kernels(self._h, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(self.obs_d.data_ptr()),
                                              ctypes.c_void_p(self.reward_d.data_ptr()),
                                              ctypes.c_void_p(self.done_d.data_ptr()), ctypes.byref(self._info),
                                              days, out.ctypes.data_as(_native.c_float_p),
                                              None if res is None else res.ctypes.data_as(_native.c_float_p),
                                              _stream_handle(self.device)), self._h)
        return (out, res) if with_resets else out

    def tables(self):
        n = ctypes.c_int32()
        irr = np.zeros(512)
        pv = np.zeros(512)
        price = np.zeros(512)   # 48 entries, 2T with the extended day (include/sng.h)
        mx = ctypes.c_double()
        pmx = ctypes.c_double()
        P = _native.c_double_p
        check(lib().sng_get_tables(self._h, irr.ctypes.data_as(P), ctypes.byref(mx), pv.ctypes.data_as(P),
                                   price.ctypes.data_as(P), ctypes.byref(pmx), ctypes.byref(n)), self._h)
        n_price = 2 * self.timesteps if self.settings.constants.get("extended_day") else 48
        return dict(irr=irr[:n.value], irr_max=mx.value, pv_power=pv[:n.value], price=price[:n_price],
                    price_max=pmx.value)


class EpisodeGraph:
    """Whole days (device-RNG reset + T fused steps, x days) captured once as a hipGraph and
    replayed; actions come from a device tensor [T, E, act_dim] reused every day."""

    def __init__(self, venv, actions, with_reset=True, days=1, day_returns=None):
        """days > 1 captures that many consecutive days (each with its reset) in one graph,
        which amortises the graph launch.  day_returns: optional device tensor [days, E] f64;
        day d's returns accumulate into row d (instead of venv.return_d).  A seed left by seed() takes effect
        here for a graph of whole days (with_reset); a steps-only graph steps the loaded day, so it is refused
        while a seed waits for the next reset."""
        if with_reset:
            venv._apply_pending_seed()
        elif venv._seeds[0] is not None:
            raise ValueError("seed() waits for the next reset: reset before capturing a steps-only graph")
        self.venv = venv
        self.days = int(days)
        self.actions = actions.contiguous()
        self.day_returns = day_returns
        dr = None
        if day_returns is not None:
            if (tuple(day_returns.shape) != (self.days, venv.num_envs) or day_returns.dtype != torch.float64
                    or day_returns.device != venv.device or not day_returns.is_contiguous()):
                raise ValueError("day_returns must be a contiguous float64 device tensor [days, num_envs]")
            dr = ctypes.c_void_p(day_returns.data_ptr())
        g = ctypes.c_void_p()
        with torch.cuda.device(venv.device):
            check(lib().sng_graph_create(venv._h, ctypes.c_void_p(self.actions.data_ptr()),
                                         ctypes.c_void_p(venv.obs_d.data_ptr()),
                                         ctypes.c_void_p(venv.reward_d.data_ptr()),
                                         ctypes.c_void_p(venv.done_d.data_ptr()), ctypes.byref(venv._info),
                                         int(with_reset), self.days, dr, ctypes.byref(g)), venv._h)
        self._g = g

    def launch(self, stream=None):
        s = _stream_handle(self.venv.device) if stream is None else ctypes.c_void_p(stream)
        check(lib().sng_graph_launch(self._g, s), self.venv._h)

    def close(self):
        if getattr(self, "_g", None):
            lib().sng_graph_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
