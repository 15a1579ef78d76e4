"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Runs only in the build container (needs /root/reference, read-only).  Nothing under
tests/ imports this module; the fixtures it writes are plain data (.npz without
pickles + .json) and are what the parity tests read on any machine.

Harness (the reference cannot be imported as shipped here):
  1. `gym` is not installed -> a stub `gym` package (Env, spaces.Box, utils.seeding,
     envs.registration) is put in sys.modules before the import.
  2. `smart_nanogrid_gym/utils/config.py:4-5` builds Windows paths -> the module globals
     are re-pointed: reads of `solar_irradiance.mat` go to the reference's files/ dir,
     every JSON write goes to a throw-away temp dir.
  3. v1 passes keyword args the current Penaliser does not accept
     (`central_management_system.py:176-179` vs `penaliser.py:95`) -> for battery variants
     `Penaliser.penalise_nanogrid_resource_issues` is wrapped to accept **kwargs and apply
     the DoD penalty only, i.e. the PenaliserOld semantics (`penaliser_old.py:98-104`).
  4. `breakpoint()` at `central_management_system.py:165` (V2X, negative demand) is replaced
     by a hook that records the event and continues (what "continue" in pdb does).

Seeding follows the reference's own contract: global `np.random.seed(s)` and
`random.seed(s)` before `reset()` (`smart_nanogrid_environment.py:349`,
`charging_station.py:214-279`).  Actions come from an independent
`np.random.default_rng(seed ^ 0x5eed)` stream, float32, uniform in the action Box,
about 20 % forced to exactly 0 and 5 % forced to exactly the upper bound.

Usage:  python tests/golden/make_golden.py        (rewrites tests/golden/*.npz, *.json)
        python tests/golden/make_golden.py eval   (only the evaluator replay cases, eval_*.npz)
"""
import builtins
import json
import os
import random
import shutil
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------------------
# harness
# ----------------------------------------------------------------------------------------
def _install_gym_stub():
    gym = types.ModuleType("gym")

    class Env:  # minimal gym.Env
        pass

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            if shape is None:
                shape = np.shape(low)
            self.shape = tuple(shape)
            self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
            self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()

    spaces = types.ModuleType("gym.spaces")
    spaces.Box = Box
    utils = types.ModuleType("gym.utils")
    seeding = types.ModuleType("gym.utils.seeding")
    utils.seeding = seeding
    envs = types.ModuleType("gym.envs")
    registration = types.ModuleType("gym.envs.registration")
    registration.registry = {}
    registration.register = lambda **kw: registration.registry.__setitem__(kw["id"], kw)
    registration.make = lambda *a, **k: None
    registration.spec = lambda *a, **k: None
    envs.registration = registration
    gym.Env, gym.spaces, gym.utils, gym.envs = Env, spaces, utils, envs
    for name, mod in {"gym": gym, "gym.spaces": spaces, "gym.utils": utils,
                      "gym.utils.seeding": seeding, "gym.envs": envs,
                      "gym.envs.registration": registration}.items():
        sys.modules[name] = mod


BREAKPOINTS = []


def import_reference(tmpdir):
    sys.dont_write_bytecode = True
    _install_gym_stub()
    sys.path.insert(0, REF)
    sys.breakpointhook = lambda *a, **k: BREAKPOINTS.append(1)
    builtins.breakpoint = lambda *a, **k: BREAKPOINTS.append(1)
    import smart_nanogrid_gym.utils.pv_system_manager as pvm
    import smart_nanogrid_gym.utils.charging_station as cs
    import smart_nanogrid_gym.utils.penaliser as pen
    import smart_nanogrid_gym.envs.smart_nanogrid_environment as envmod

    pvm.data_files_directory_path = os.path.join(REF, "smart_nanogrid_gym", "files") + "/"
    cs.data_files_directory_path = tmpdir + "/"
    envmod.data_files_directory_path = tmpdir + "/"
    envmod.solvers_files_directory_path = tmpdir + "/"
    os.makedirs(os.path.join(tmpdir, "RL"), exist_ok=True)

    def dod_only(self, current_state_of_charge=None, depth_of_discharge=None, **_ignored):
        self.penalise_battery_state_below_depth_of_discharge(current_state_of_charge, depth_of_discharge)

    pen.Penaliser.penalise_nanogrid_resource_issues = dod_only
    return envmod.SmartNanogridEnv


# ----------------------------------------------------------------------------------------
# recording
# ----------------------------------------------------------------------------------------
RESULT_KEYS = {
    "grid_power": "Grid power",
    "p_charge": "Total charging power",
    "p_discharge": "Total discharging power",
    "bess_soc": "Battery state of charge",
    "pen_vehicle": "Total vehicle penalty",
    "pen_battery": "Total battery penalty",
    "grid_cost": "Grid energy cost",
    "total_cost": "Total cost",
    "solar_power": "Utilized solar energy",
    "bess_power": "Battery power value",
    "bess_calc_power": "Battery calculated power value",
    "nonexistent": "DisCharging nonexistent vehicles penalty",
    "bess_initial_soc": "Initial battery state of charge",
}

VMAX = 8  # padded per-charger arrival/departure lists


def make_actions(rng, space, n_steps, zero_frac=0.2, one_frac=0.05):
    low = space.low.astype(np.float64)
    high = space.high.astype(np.float64)
    a = rng.uniform(low, high, size=(n_steps,) + space.shape).astype(np.float32)
    r = rng.random(a.shape)
    a[r < zero_frac] = 0.0
    hi = np.broadcast_to(space.high, a.shape)
    sel = (r >= zero_frac) & (r < zero_frac + one_frac)
    a[sel] = hi[sel]
    return a


def run_case(Env, name, kwargs, seed, n_episodes, act_override=None, persist_between=True):
    np.random.seed(seed)
    random.seed(seed)
    env = Env(**kwargs)
    cms = env.central_management_system
    T = int(24 / env.TIME_INTERVAL)
    N = env.NUMBER_OF_CHARGERS
    act_rng = np.random.default_rng(seed ^ 0x5EED)

    captured = {}
    orig = cms.simulate

    def spy(timestep, actions, ratio):
        res = orig(timestep, actions, ratio)
        captured["res"] = res
        return res

    cms.simulate = spy

    rec = {k: [] for k in ["obs_reset", "obs", "reward", "done", "actions", "ratio", "bess_soc_reset",
                           "soc0", "occ", "cap", "req", "arrivals", "departures", "charger_power",
                           "breakpoint"] + list(RESULT_KEYS)}
    for ep in range(n_episodes):
        bess_before = cms.battery_system.current_state_of_charge if cms.battery_system else 0.0
        obs0, info = env.reset()
        gv = cms.charging_station.generated_initial_values
        rec["obs_reset"].append(np.asarray(obs0, np.float32))
        rec["ratio"].append(env.random_pv_shift_ratio)
        rec["bess_soc_reset"].append(bess_before)
        rec["soc0"].append(np.array(gv["SOC"], np.float64))
        rec["occ"].append(np.array(gv["Charger_occupancy"], np.float64))
        rec["cap"].append(np.array(gv["Vehicle_capacities"], np.float64))
        rec["req"].append(np.array(gv["Requested_SOC"], np.float64))
        arr = np.full((N, VMAX), -1, np.int64)
        dep = np.full((N, VMAX), -1, np.int64)
        for c in range(N):
            arr[c, :len(gv["Arrivals"][c])] = gv["Arrivals"][c]
            dep[c, :len(gv["Departures"][c])] = gv["Departures"][c]
        rec["arrivals"].append(arr)
        rec["departures"].append(dep)
        acts = make_actions(act_rng, env.action_space, T) if act_override is None else act_override(act_rng, env, T)
        rec["actions"].append(acts)
        ep_rows = {k: [] for k in ["obs", "reward", "done", "charger_power", "breakpoint"] + list(RESULT_KEYS)}
        for t in range(T):
            del BREAKPOINTS[:]
            obs, reward, term, trunc, info = env.step(acts[t].copy())
            r = captured["res"]
            ep_rows["obs"].append(np.asarray(obs, np.float32))
            ep_rows["reward"].append(float(reward))
            ep_rows["done"].append(bool(term))
            ep_rows["charger_power"].append(np.array(r["Charger power values"], np.float64))
            ep_rows["breakpoint"].append(len(BREAKPOINTS))
            for k, rk in RESULT_KEYS.items():
                ep_rows[k].append(float(r[rk]))
        for k, v in ep_rows.items():
            rec[k].append(np.array(v))
    out = {k: np.array(v) for k, v in rec.items()}
    meta = dict(name=name, kwargs=kwargs, seed=seed, n_episodes=n_episodes, T=T, N=N,
                obs_dim=int(env.observation_space.shape[0]), act_dim=int(env.action_space.shape[0]),
                act_low=env.action_space.low.tolist(), act_high=env.action_space.high.tolist())
    return out, meta


def run_evaluator_case(Env, name, kwargs, seed, n_models, n_episodes, act_override=None):
    """The loop of solvers/evaluator.py:88-101 on one env (the evaluator shares one env per variant):
    per episode, model 0's reset generates the day (generate_new_initial_values=True, which writes
    initial_values.json, charging_station.py:185-186) and every further model replays it
    (generate_new_initial_values=False -> load_initial_values, :119-136: Requested_SOC is not restored,
    the PV ratio is redrawn, smart_nanogrid_environment.py:349).  Model m's actions come from its own
    stream default_rng((seed ^ 0x5EED) + 101 * m), one day of actions per episode."""
    np.random.seed(seed)
    random.seed(seed)
    env = Env(**kwargs)
    cms = env.central_management_system
    T = int(24 / env.TIME_INTERVAL)
    N = env.NUMBER_OF_CHARGERS
    act_rngs = [np.random.default_rng((seed ^ 0x5EED) + 101 * m) for m in range(n_models)]
    captured = {}
    orig = cms.simulate

    def spy(timestep, actions, ratio):
        res = orig(timestep, actions, ratio)
        captured["res"] = res
        return res

    cms.simulate = spy
    rec = {k: [] for k in ["obs_reset", "obs", "reward", "done", "actions", "ratio", "bess_soc_reset", "generated",
                           "soc0", "occ", "cap", "req", "arrivals", "departures"] + list(RESULT_KEYS)}
    for ep in range(n_episodes):
        for m in range(n_models):
            generate = m == 0
            bess_before = cms.battery_system.current_state_of_charge if cms.battery_system else 0.0
            obs0, _ = env.reset(generate_new_initial_values=generate, algorithm_used="PPO",
                                environment_mode="evaluation")
            gv = cms.charging_station.generated_initial_values
            rec["obs_reset"].append(np.asarray(obs0, np.float32))
            rec["ratio"].append(env.random_pv_shift_ratio)
            rec["bess_soc_reset"].append(bess_before)
            rec["generated"].append(generate)
            rec["soc0"].append(np.array(gv["SOC"], np.float64))
            rec["occ"].append(np.array(gv["Charger_occupancy"], np.float64))
            rec["cap"].append(np.array(gv["Vehicle_capacities"], np.float64))
            rec["req"].append(np.array(gv["Requested_SOC"], np.float64))
            arr = np.full((N, VMAX), -1, np.int64)
            dep = np.full((N, VMAX), -1, np.int64)
            for c in range(N):
                arr[c, :len(gv["Arrivals"][c])] = gv["Arrivals"][c]
                dep[c, :len(gv["Departures"][c])] = gv["Departures"][c]
            rec["arrivals"].append(arr)
            rec["departures"].append(dep)
            rng = act_rngs[m]
            acts = make_actions(rng, env.action_space, T) if act_override is None else act_override(rng, env, T)
            rec["actions"].append(acts)
            rows = {k: [] for k in ["obs", "reward", "done"] + list(RESULT_KEYS)}
            for t in range(T):
                obs, reward, term, trunc, info = env.step(acts[t].copy())
                r = captured["res"]
                rows["obs"].append(np.asarray(obs, np.float32))
                rows["reward"].append(float(reward))
                rows["done"].append(bool(term))
                for k, rk in RESULT_KEYS.items():
                    rows[k].append(float(r[rk]))
            for k, v in rows.items():
                rec[k].append(np.array(v))
    out = {k: np.array(v) for k, v in rec.items()}
    meta = dict(name=name, kwargs=kwargs, seed=seed, n_models=n_models, n_episodes=n_episodes, T=T, N=N,
                obs_dim=int(env.observation_space.shape[0]), act_dim=int(env.action_space.shape[0]))
    return out, meta


def base_kwargs(**over):
    kw = dict(price_model=0, number_of_chargers=10, pv_system_available_in_model=True,
              battery_system_available_in_model=True, vehicle_to_everything=False,
              enable_different_vehicle_battery_capacities=True, enable_requested_state_of_charge=False,
              algorithm_used="PPO", environment_mode="training", time_interval="1h",
              charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    kw.update(over)
    return kw


def heavy_discharge(rng, env, T):
    """Battery action mostly -1 so the BESS hits the over-discharge clamp and DoD penalty."""
    a = make_actions(rng, env.action_space, T)
    a[:, -1] = np.where(rng.random(T) < 0.8, np.float32(-1.0), a[:, -1])
    return a


def heavy_v2x_discharge(rng, env, T):
    """V2X: push EVs to discharge (negative demand -> breakpoint path, inverted-flag quirk)."""
    a = make_actions(rng, env.action_space, T)
    n = env.NUMBER_OF_CHARGERS
    a[:, :n] = np.where(rng.random((T, n)) < 0.7, -np.abs(a[:, :n]), a[:, :n])
    return a


CASES = [
    # name, kwargs, seed, episodes, action override
    ("bpv_sparse_n1", base_kwargs(number_of_chargers=1), 11, 4, None),
    ("bpv_sparse_n4", base_kwargs(number_of_chargers=4), 12, 4, None),
    ("bpv_sparse_n10", base_kwargs(), 13, 4, None),
    ("bpv_sparse_n50", base_kwargs(number_of_chargers=50), 14, 3, None),
    ("bpv_nopen_n10", base_kwargs(vehicle_uncharged_penalty_mode="no_penalty"), 21, 3, None),
    ("bpv_ondep_n10", base_kwargs(vehicle_uncharged_penalty_mode="on_departure"), 22, 3, None),
    ("bpv_dense_n10", base_kwargs(vehicle_uncharged_penalty_mode="dense"), 23, 3, None),
    ("basic_sparse_n10", base_kwargs(pv_system_available_in_model=False,
                                     battery_system_available_in_model=False), 31, 3, None),
    ("pv_sparse_n10", base_kwargs(battery_system_available_in_model=False), 32, 3, None),
    ("bess_sparse_n10", base_kwargs(pv_system_available_in_model=False), 33, 3, None),
    ("bpv_req_n10", base_kwargs(enable_requested_state_of_charge=True), 41, 3, None),
    ("bpv_samecap_n10", base_kwargs(enable_different_vehicle_battery_capacities=False), 42, 3, None),
    ("bpv_2h_n10", base_kwargs(time_interval="2h"), 43, 3, None),
    ("bpv_price1_n4", base_kwargs(number_of_chargers=4, price_model=1), 51, 2, None),
    ("bpv_price2_n4", base_kwargs(number_of_chargers=4, price_model=2), 52, 2, None),
    ("bpv_price3_n4", base_kwargs(number_of_chargers=4, price_model=3), 53, 2, None),
    ("bpv_price4_n4", base_kwargs(number_of_chargers=4, price_model=4), 54, 2, None),
    ("bpv_dod_n10", base_kwargs(), 61, 4, heavy_discharge),
    ("v2x_basic_n10", base_kwargs(vehicle_to_everything=True, pv_system_available_in_model=False,
                                  battery_system_available_in_model=False), 71, 3, heavy_v2x_discharge),
    ("v2x_bpv_n10", base_kwargs(vehicle_to_everything=True), 72, 3, heavy_v2x_discharge),
    ("bpv_dense_req_n50", base_kwargs(number_of_chargers=50, vehicle_uncharged_penalty_mode="dense",
                                      enable_requested_state_of_charge=True), 81, 2, None),
]


# solvers/evaluator.py:88-101 replays (reset True, then False for the other models), per episode
EVAL_CASES = [
    # name, kwargs, seed, models, episodes, action override
    ("eval_replay_req_dense_n10", base_kwargs(enable_requested_state_of_charge=True,
                                              vehicle_uncharged_penalty_mode="dense"), 91, 3, 2, None),
    ("eval_replay_sparse_n4", base_kwargs(number_of_chargers=4), 92, 3, 2, None),
    ("eval_replay_dod_n10", base_kwargs(), 93, 3, 2, heavy_discharge),
]


def tables_fixture(Env, tmp):
    """Derived per-dt constant tables straight from the reference objects."""
    out = {}
    for ti in ["1h", "2h", "15min", "30min"]:
        np.random.seed(0)
        random.seed(0)
        try:
            env = Env(**base_kwargs(time_interval=ti))
        except Exception as e:  # the reference cannot run every dt
            out[f"{ti}_error"] = np.array(str(type(e).__name__))
            continue
        cms = env.central_management_system
        pv = cms.pv_system_manager
        out[f"{ti}_irr"] = np.array(pv.solar_irradiance_2[0], np.float64)
        out[f"{ti}_irr_max"] = np.array(pv.max_radiation, np.float64)
        out[f"{ti}_pv_power"] = np.array(pv.available_solar_power[0], np.float64)
        out[f"{ti}_price"] = np.array(cms.accountant.energy_price[0], np.float64)
        out[f"{ti}_price_max"] = np.array(cms.accountant.energy_price_max, np.float64)
    for pm in range(5):
        env = Env(**base_kwargs(price_model=pm))
        out[f"price_model{pm}"] = np.array(env.central_management_system.accountant.energy_price[0], np.float64)
    return out


def main_eval(Env):
    index = []
    for name, kw, seed, models, eps, override in EVAL_CASES:
        out, meta = run_evaluator_case(Env, name, kw, seed, models, eps, override)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        index.append(meta)
        print(f"{name}: N={meta['N']} models={models} episodes={eps} "
              f"returns={[round(float(r.sum()), 4) for r in out['reward']]}")
    with open(os.path.join(HERE, "eval_cases.json"), "w") as fp:
        json.dump(index, fp, indent=1)


def main():
    tmp = tempfile.mkdtemp(prefix="sng_golden_")
    if sys.argv[1:] == ["eval"]:   # only the evaluator replay cases
        try:
            main_eval(import_reference(tmp))
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    try:
        Env = import_reference(tmp)
        main_eval(Env)
        index = []
        for name, kw, seed, eps, override in CASES:
            out, meta = run_case(Env, name, kw, seed, eps, override)
            np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
            index.append(meta)
            print(f"{name}: N={meta['N']} T={meta['T']} episodes={eps} "
                  f"return[0]={out['reward'][0].sum():.6f} breakpoints={int(out['breakpoint'].sum())}")
        with open(os.path.join(HERE, "cases.json"), "w") as fp:
            json.dump(index, fp, indent=1)
        np.savez_compressed(os.path.join(HERE, "tables.npz"), **tables_fixture(Env, tmp))
        # per-minute irradiance: the product's PV input data (derived, raw little-endian f64)
        from scipy.io import loadmat
        irr = loadmat(os.path.join(REF, "smart_nanogrid_gym", "files", "solar_irradiance.mat"))["irradiance"]
        irr = np.ascontiguousarray(irr[:, 0], dtype="<f8")
        data_dir = os.path.join(HERE, "..", "..", "smart-nanogrid-gym_amd", "smart_nanogrid_gym", "data")
        irr.tofile(os.path.join(data_dir, "solar_irradiance_1min.f64"))
        # recorded PPO episodes shipped inside the reference (known-answer trajectories)
        for sub in ["single_prediction_files", "training_files"]:
            for suffix in ["initial_values", "prediction_results"]:
                src = os.path.join(REF, "solvers", "RL", sub, f"PPO-b-pv-bounded-sparse-4ch-1h-{suffix}.json")
                shutil.copyfile(src, os.path.join(HERE, "kat", f"{sub}-{suffix}.json"))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
