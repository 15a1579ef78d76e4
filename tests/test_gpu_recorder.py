"""GPU: the day recorder (28-key prediction_results.json / initial_values.json, reference
smart_nanogrid_environment.py:239-309 and charging_station.py:164-191) and the timeline decode
behind it (sng_get_scenario).

Pinned three ways: the reference's own recorded PPO days (tests/golden/kat: every key, the
file names and the initial values), the CPU oracle's arrays and per-step results for
reference-RNG days, and a decode -> reset_from_initial_values round trip for device-RNG days
(the re-injected day must step bit for bit like the original).  Tolerance: 1e-12 relative on
floating-point results against the reference's numbers (its libm pow differs by one ulp on
~0.1 % of inputs), bit-exact against the oracle in x*x mode and for SoC / scenario arrays.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle as O
from golden_util import kat

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smart_nanogrid_gym import DayRecorder, SmartNanogridEnv, SmartNanogridVecEnv  # noqa: E402
from smart_nanogrid_gym.recorder import RESULT_KEYS  # noqa: E402

ORACLE_INFO = {"grid_power": "Grid_power", "total_cost": "Total_cost", "grid_cost": "Grid_energy_cost",
               "p_charge": "Total_charging_power", "p_discharge": "Total_discharging_power",
               "bess_soc": "Battery_state_of_charge", "pen_vehicle": "Total_vehicle_penalties",
               "pen_battery": "Total_battery_penalties", "solar_power": "Utilized_solar_energy",
               "bess_power": "Battery_power_value", "bess_calc_power": "Battery_calculated_power_value",
               "nonexistent": "DisCharging_nonexistent_vehicles_penalties"}


def close(a, b, tol=1e-12):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return a.shape == b.shape and bool(np.all(np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b))))


@pytest.fixture(scope="module", autouse=True)
def _square_mode():
    O.lib().orc_set_square_mode.argtypes = [ctypes.c_int]
    O.lib().orc_set_square_mode(1)   # the GPU squares with x*x (test_gpu_parity.py)
    yield
    O.lib().orc_set_square_mode(0)


@pytest.mark.parametrize("sub,mode", [("single_prediction_files", "prediction"), ("training_files", "training")])
def test_recorder_reproduces_recorded_ppo_day(sub, mode, tmp_path):
    """Replay the reference's recorded day; the files written must be the reference's files."""
    k = kat(sub)
    venv = SmartNanogridVecEnv(1, number_of_chargers=k["N"], time_interval="1h", charging_mode="bounded",
                               vehicle_uncharged_penalty_mode="sparse", numpy_legacy_promotion=True,
                               grid_cost_weight=0.8, algorithm_used="PPO", environment_mode=mode)
    rec = DayRecorder(venv, [0], directory=str(tmp_path))
    venv.set_battery_state_of_charge(k["bess_soc0"])
    venv.reset_from_initial_values(k["iv"], k["ratio"], restore_requested_soc=True)
    for t in range(24):
        venv.step_tensors(torch.from_numpy(k["actions"][t][None]).to(venv.device))
    stem = os.path.join(str(tmp_path), sub, "PPO-b-pv-bounded-sparse-4ch-1h")
    with open(stem + "-prediction_results.json") as fp:
        pr = json.load(fp)
    with open(stem + "-initial_values.json") as fp:
        iv = json.load(fp)
    ref = k["pr"]
    assert list(pr) == list(ref) == RESULT_KEYS
    for key in RESULT_KEYS:
        assert close(pr[key], ref[key]), key
    for key in ("SOC", "Charger_actions", "Battery_action", "Available_solar_energy", "Battery_state_of_charge"):
        assert pr[key] == ref[key], key        # bit for bit
    assert iv == k["iv"]
    venv.close()


CONFIGS = {
    "bpv_sparse_n10": dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded",
                           vehicle_uncharged_penalty_mode="sparse"),
    "bpv_dense_req_n10": dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded",
                              vehicle_uncharged_penalty_mode="dense", enable_requested_state_of_charge=True),
    "v2x_bpv_ondep_n7": dict(number_of_chargers=7, time_interval="1h", charging_mode="bounded",
                             vehicle_uncharged_penalty_mode="on_departure", vehicle_to_everything=True),
    "basic_2h_n4": dict(number_of_chargers=4, time_interval="2h", charging_mode="bounded",
                        vehicle_uncharged_penalty_mode="sparse", pv_system_available_in_model=False,
                        battery_system_available_in_model=False),
}


@pytest.mark.parametrize("name", list(CONFIGS))
def test_recorder_matches_oracle_reference_rng(name):
    """Reference-RNG days: initial values = the oracle's generated arrays, 'SOC' = the oracle's
    arrays after the day, per-step results = the oracle's results dict."""
    kw = CONFIGS[name]
    E, seed, ids = 64, 4242, [0, 17, 63]
    venv = SmartNanogridVecEnv(E, seed=seed, rng="reference", **kw)
    rec = DayRecorder(venv, ids, keep_history=True)
    cfg = O.OracleConfig(**kw)
    envs = {i: O.OracleEnv(cfg, seed + i) for i in ids}
    rng = np.random.default_rng(7)
    N, S = cfg.N, cfg.slots
    for day in range(2):
        if day == 0:
            venv.reset()
        for i, e in envs.items():
            e.reset()
            sc = e.scenario(vmax=16)
            iv = rec.initial_values(i)
            assert iv["SOC"] == sc["soc"].tolist(), (day, i)
            assert iv["Charger_occupancy"] == sc["occ"].tolist()
            assert iv["Vehicle_capacities"] == sc["cap"].tolist()
            assert iv["Requested_SOC"] == sc["req"].tolist()
            assert iv["Arrivals"] == [[a for a in row if a >= 0] for row in sc["arrivals"].tolist()]
            assert iv["Departures"] == [[a for a in row if a >= 0] for row in sc["departures"].tolist()]
        infos = {i: [] for i in ids}
        acts = []
        for t in range(cfg.T):
            a = rng.uniform(venv.action_space.low, venv.action_space.high, (E, venv.act_dim)).astype(np.float32)
            a[rng.random(a.shape) < 0.2] = 0
            acts.append(a)
            for i, e in envs.items():
                infos[i].append(e.step(a[i])[3])
            venv.step(a)   # auto-resets after the last step: the recorder has closed the day by then
        for i, e in envs.items():
            pr, _ = rec.last[i]
            assert list(pr) == RESULT_KEYS
            assert pr["SOC"] == e.scenario()["soc"].tolist(), (day, i)
            for ok, rk in ORACLE_INFO.items():
                assert pr[rk] == [inf[ok] for inf in infos[i]], (day, i, rk)
            assert pr["Charger_actions"] == [acts[t][i][:N].tolist() for t in range(cfg.T)]
            for t in range(cfg.T):
                pw = np.array(pr["Charger_power_values"][t])
                assert pw.shape == (N,)
                assert O.pairwise_sum(pw[pw > 0]) == pr["Total_charging_power"][t]
                assert O.pairwise_sum(pw[pw < 0]) == pr["Total_discharging_power"][t]
            assert len(pr["SOC"]) == N and all(len(r) == S for r in pr["SOC"])
    assert len(rec.history) == 2 * len(ids)
    venv.close()


@pytest.mark.parametrize("N,req,dt", [(10, False, "1h"), (10, True, "1h"), (33, True, "1h"), (128, False, "1h"),
                                      (10, True, "30min"), (16, False, "20min"), (4, True, "2h")])
def test_device_day_decode_round_trip(N, req, dt):
    """Device-RNG days decoded to the reference layout and re-injected step bit for bit like the original.
    N = 33 and 128 (the maximum) take the generic step kernel and the separate t = 0 observation launch;
    20 min (dt = 1/3, not a power of two) takes the division path of the step."""
    kw = dict(number_of_chargers=N, time_interval=dt, charging_mode="bounded",
              vehicle_uncharged_penalty_mode="dense" if req else "sparse", enable_requested_state_of_charge=req)
    if dt.endswith("min"):
        kw["extended_day"] = True   # sub-hour days need the build-defined extension (section 5.4)
    E = 256
    a_dev = SmartNanogridVecEnv(E, seed=99, rng="device", **kw)
    b_inj = SmartNanogridVecEnv(E, seed=0, **kw)
    obs_a = a_dev.reset_tensors().cpu().numpy().copy()
    ivs, ratios = zip(*[a_dev.get_scenario(i) for i in range(E)])
    min_stay = a_dev.timesteps // 6   # the device generator's process: every vehicle stays >= 4 h
    for iv in ivs:
        for arr, dep in zip(iv["Arrivals"], iv["Departures"]):
            assert all(d - a >= min_stay for a, d in zip(arr, dep))
    b_inj.set_battery_state_of_charge(a_dev.battery_state_of_charge())
    obs_b = b_inj.reset_from_initial_values(list(ivs), np.array(ratios), restore_requested_soc=True)
    np.testing.assert_array_equal(obs_a, obs_b)
    rng = np.random.default_rng(3)
    for t in range(a_dev.timesteps):
        a = torch.from_numpy(rng.uniform(-1, 1, (E, a_dev.act_dim)).astype(np.float32)).to(a_dev.device)
        # chargers in their Box [0, 1]; the BESS action keeps its negative half (discharge, over-discharge clamp)
        a[:, :N] = torch.where(a[:, :N] < 0, torch.zeros_like(a[:, :N]), a[:, :N])
        oa, ra, _ = a_dev.step_tensors(a)
        ob, rb, _ = b_inj.step_tensors(a)
        assert torch.equal(oa, ob), t
        assert torch.equal(ra, rb), t
    a_dev.close()
    b_inj.close()


def test_single_env_writes_reference_files(tmp_path):
    """SmartNanogridEnv(results_directory=...) writes a file pair at each day end, as the reference does."""
    env = SmartNanogridEnv(number_of_chargers=4, time_interval="1h", charging_mode="bounded",
                           vehicle_uncharged_penalty_mode="sparse", algorithm_used="DDPG",
                           environment_mode="evaluation", results_directory=str(tmp_path), seed=5)
    env.reset()
    for _ in range(24):
        env.step(env.action_space.sample() * 0)
    stem = os.path.join(str(tmp_path), "evaluation_files", "DDPG-b-pv-bounded-sparse-4ch-1h")
    with open(stem + "-prediction_results.json") as fp:
        pr = json.load(fp)
    with open(stem + "-initial_values.json") as fp:
        iv = json.load(fp)
    assert list(pr) == RESULT_KEYS and len(pr["Grid_power"]) == 24
    assert set(iv) == {"SOC", "Arrivals", "Departures", "Charger_occupancy", "Vehicle_capacities", "Requested_SOC"}
    assert all(v == 0.0 for v in pr["Charger_power_values"][0])   # zero actions
    env.close()
