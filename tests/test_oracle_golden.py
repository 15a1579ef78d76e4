"""The CPU oracle against outputs of the reference itself (tests/golden, made by make_golden.py)
and against the reference's recorded PPO episodes (tests/golden/kat)."""
import numpy as np
import pytest

import oracle as O
from golden_util import case, cases, eval_case, eval_cases, kat, load_case

CASES = [m["name"] for m in cases()]
SCALARS = ["grid_power", "p_charge", "p_discharge", "bess_soc", "pen_vehicle", "pen_battery", "grid_cost",
           "total_cost", "solar_power", "bess_power", "bess_calc_power", "nonexistent", "bess_initial_soc"]


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_bit_exact(name):
    meta, d = case(name)
    cfg = O.OracleConfig(**meta["kwargs"])
    env = O.OracleEnv(cfg, meta["seed"])
    for ep in range(meta["n_episodes"]):
        obs = env.reset()
        np.testing.assert_array_equal(obs, d["obs_reset"][ep])
        assert env.ratio == d["ratio"][ep]
        sc = env.scenario()
        np.testing.assert_array_equal(sc["soc"], d["soc0"][ep])
        np.testing.assert_array_equal(sc["occ"], d["occ"][ep])
        np.testing.assert_array_equal(sc["cap"], d["cap"][ep])
        np.testing.assert_array_equal(sc["req"], d["req"][ep])
        np.testing.assert_array_equal(sc["arrivals"], d["arrivals"][ep])
        np.testing.assert_array_equal(sc["departures"], d["departures"][ep])
        for t in range(meta["T"]):
            obs, r, done, info = env.step(d["actions"][ep][t])
            np.testing.assert_array_equal(obs, d["obs"][ep][t])
            assert r == d["reward"][ep][t], (ep, t)
            assert done == bool(d["done"][ep][t])
            assert info["breakpoint"] == int(d["breakpoint"][ep][t] > 0)
            for k in SCALARS:
                assert info[k] == d[k][ep][t], (k, ep, t)


def test_tables_match_reference():
    t = np.load(f"{O.HERE}/../tests/golden/tables.npz")
    for ti in ["1h", "2h", "15min", "30min"]:
        cfg = O.OracleConfig(number_of_chargers=2, time_interval=ti)
        tb = cfg.tables()
        np.testing.assert_array_equal(tb["irr"], t[f"{ti}_irr"])
        np.testing.assert_array_equal(tb["pv_power"], t[f"{ti}_pv_power"])
        assert tb["irr_max"] == t[f"{ti}_irr_max"]
        np.testing.assert_array_equal(tb["price"], t[f"{ti}_price"])
        assert tb["price_max"] == t[f"{ti}_price_max"]
    for pm in range(5):
        cfg = O.OracleConfig(number_of_chargers=2, price_model=pm)
        np.testing.assert_array_equal(cfg.tables()["price"], t[f"price_model{pm}"])


@pytest.mark.parametrize("sub", ["single_prediction_files", "training_files"])
def test_oracle_replays_recorded_ppo_episode(sub):
    """Recorded with NumPy 1.24 (float64 EV power) and a 0.8 grid-cost weight: with those two
    settings the replay reproduces every recorded series exactly."""
    k = kat(sub)
    iv, pr = k["iv"], k["pr"]
    cfg = O.OracleConfig(number_of_chargers=k["N"], time_interval="1h", vehicle_uncharged_penalty_mode="sparse",
                         numpy_legacy_promotion=True, grid_cost_weight=0.8)
    env = O.OracleEnv(cfg, 0)
    env.bess_soc = k["bess_soc0"]
    env.load(iv["SOC"], iv["Charger_occupancy"], iv["Vehicle_capacities"], iv["Requested_SOC"],
             k["arrivals"], k["departures"], k["ratio"])
    pairs = [("grid_power", "Grid_power"), ("bess_soc", "Battery_state_of_charge"),
             ("pen_vehicle", "Total_vehicle_penalties"), ("total_cost", "Total_cost"),
             ("grid_cost", "Grid_energy_cost"), ("p_charge", "Total_charging_power"),
             ("p_discharge", "Total_discharging_power"), ("solar_power", "Utilized_solar_energy"),
             ("bess_power", "Battery_power_value")]
    for t in range(24):
        _, r, done, info = env.step(k["actions"][t])
        for ok, rk in pairs:
            assert info[ok] == pr[rk][t], (ok, t)
        assert done == (t == 23)
    np.testing.assert_array_equal(env.scenario(k["arrivals"].shape[1])["soc"], np.array(pr["SOC"]))


@pytest.mark.parametrize("sub", ["single_prediction_files", "training_files"])
def test_oracle_numpy2_promotion_close_to_recording(sub):
    """Default (NumPy 2, float32 EV power) differs from the NumPy 1.24 recording by < 2e-6."""
    k = kat(sub)
    iv, pr = k["iv"], k["pr"]
    cfg = O.OracleConfig(number_of_chargers=k["N"], time_interval="1h", grid_cost_weight=0.8)
    env = O.OracleEnv(cfg, 0)
    env.bess_soc = k["bess_soc0"]
    env.load(iv["SOC"], iv["Charger_occupancy"], iv["Vehicle_capacities"], iv["Requested_SOC"],
             k["arrivals"], k["departures"], k["ratio"])
    for t in range(24):
        _, r, _, info = env.step(k["actions"][t])
        assert abs(info["grid_power"] - pr["Grid_power"][t]) < 2e-6
        assert abs(info["total_cost"] - pr["Total_cost"][t]) < 2e-6


@pytest.mark.parametrize("name", [m["name"] for m in eval_cases()])
def test_oracle_replays_like_the_reference_evaluator(name):
    """solvers/evaluator.py:88-101 on the reference: reset(generate_new_initial_values=True) for the first
    model of an episode, False for the others (load_initial_values: same vehicles, Requested_SOC not
    restored, a new PV ratio).  The oracle's replay matches it bit for bit, per model and episode."""
    meta, d = eval_case(name)
    cfg = O.OracleConfig(**meta["kwargs"])
    env = O.OracleEnv(cfg, meta["seed"])
    k = 0
    for ep in range(meta["n_episodes"]):
        for m in range(meta["n_models"]):
            assert bool(d["generated"][k]) == (m == 0)
            obs = env.reset() if m == 0 else env.replay()
            np.testing.assert_array_equal(obs, d["obs_reset"][k])
            assert env.ratio == d["ratio"][k]
            assert env.bess_soc == d["bess_soc_reset"][k]
            for t in range(meta["T"]):
                obs, r, done, info = env.step(d["actions"][k][t])
                np.testing.assert_array_equal(obs, d["obs"][k][t])
                assert r == d["reward"][k][t], (ep, m, t)
                for key in SCALARS:
                    assert info[key] == d[key][k][t], (key, ep, m, t)
                if m > 0:   # a replayed day never penalises a vehicle (Requested_SOC = 0)
                    assert info["pen_vehicle"] == 0.0
            k += 1
    # the generated days penalise (dense / sparse modes), so the replay's zero penalty is a real difference
    assert d["pen_vehicle"][0].sum() > 0
