"""CPU checks of the day recorder's host logic against the reference's recorded files
(tests/golden/kat): key set and order, the PV energy table, the file naming.  The recorder's
device side is covered by tests/test_gpu_recorder.py."""
import types

import numpy as np
import pytest

import oracle as O
from golden_util import kat

pytest.importorskip("torch")
from smart_nanogrid_gym import EnvSettings  # noqa: E402
from smart_nanogrid_gym.recorder import RESULT_KEYS, DayRecorder, available_solar_energy  # noqa: E402


@pytest.mark.parametrize("sub", ["single_prediction_files", "training_files"])
def test_result_keys_are_the_reference_keys(sub):
    assert RESULT_KEYS == list(kat(sub)["pr"])
    assert len(RESULT_KEYS) == 28


@pytest.mark.parametrize("sub", ["single_prediction_files", "training_files"])
def test_available_solar_energy_bit_exact(sub):
    """pv_system_manager.py:67-73 on the per-step irradiance table (oracle tables, pinned
    against the reference by test_tables_match_reference)."""
    cfg = O.OracleConfig(number_of_chargers=4, time_interval="1h")
    irr = cfg.tables()["irr"][:48]
    assert available_solar_energy(irr) == kat(sub)["pr"]["Available_solar_energy"]


def test_never_computed_penalties_are_zero_in_the_recording():
    """The reference never assigns these (penaliser.py): always 0.0 in its files."""
    pr = kat("single_prediction_files")["pr"]
    for key in ("Low_resource_utilisation_penalties", "Battery_overcharging_penalties",
                "Battery_over_discharging_penalties", "Needlessly_charged_vehicle_penalties",
                "Overcharged_vehicle_penalties", "Over_discharged_vehicle_penalties"):
        assert all(v == 0.0 for v in pr[key])
    assert pr["Battery_SOC_below_DoD_penalties"] == pr["Total_battery_penalties"]
    assert pr["Insufficiently_charged_vehicle_penalties"] == pr["Total_vehicle_penalties"]
    assert pr["Grid_energy"] == [g * 1.0 for g in pr["Grid_power"]]


@pytest.mark.parametrize("kw,stem", [
    (dict(algorithm_used="PPO", number_of_chargers=4, time_interval="1h", charging_mode="bounded",
          vehicle_uncharged_penalty_mode="sparse"), "PPO-b-pv-bounded-sparse-4ch-1h"),
    (dict(algorithm_used="DDPG", number_of_chargers=10, time_interval="15min", charging_mode="bounded",
          vehicle_uncharged_penalty_mode="dense", vehicle_to_everything=True), "DDPG-v2x-b-pv-bounded-dense-10ch-15min"),
    (dict(algorithm_used="A2C", number_of_chargers=3, time_interval="2h", charging_mode="bounded",
          vehicle_uncharged_penalty_mode="on_departure", pv_system_available_in_model=False),
     "A2C-basic-bounded-on_departure-3ch-2h"),
])
def test_file_names_follow_the_reference(kw, stem):
    """smart_nanogrid_environment.py:280-303"""
    rec = DayRecorder.__new__(DayRecorder)
    rec.venv = types.SimpleNamespace(settings=EnvSettings(**kw))
    rec.env_ids = [0]
    assert rec.file_stem(0) == stem
    rec.env_ids = [0, 3]
    assert rec.file_stem(3) == stem + "-env3"


def test_recorded_soc_is_the_oracle_day_end_array():
    """'SOC' in the recorded file is the charger arrays after the day (charger.py:37-56 rewrite
    SOC[c, t] at every occupied step): the oracle's arrays after replaying the day."""
    k = kat("training_files")
    iv = k["iv"]
    cfg = O.OracleConfig(number_of_chargers=k["N"], time_interval="1h", numpy_legacy_promotion=True,
                         grid_cost_weight=0.8)
    env = O.OracleEnv(cfg, 0)
    env.bess_soc = k["bess_soc0"]
    env.load(iv["SOC"], iv["Charger_occupancy"], iv["Vehicle_capacities"], iv["Requested_SOC"],
             k["arrivals"], k["departures"], k["ratio"])
    for t in range(24):
        env.step(k["actions"][t])
    assert env.scenario(k["arrivals"].shape[1])["soc"].tolist() == k["pr"]["SOC"]
    assert np.array(k["pr"]["SOC"]).shape == (k["N"], 25)
