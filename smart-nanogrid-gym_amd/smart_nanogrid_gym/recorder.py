"""Per-day result files of the reference, for selected envs of a batch.

The reference env records every step's results dict and, when a day ends, writes
`<ALGO>-<variant>-<charging mode>-<penalty mode>-<N>ch-<interval>-prediction_results.json`
(28 keys, SmartNanogridEnv.__save_prediction_results, smart_nanogrid_environment.py:239-309)
and the day's `...-initial_values.json` (ChargingStation.save_initial_values_to_json_file,
charging_station.py:187-191) under solvers/RL/<training|evaluation|single_prediction>_files/.

DayRecorder does the same for the env indices it is given: the step kernel writes the
per-env diagnostics plus the per-charger power and SoC into device arrays (SngInfo), the
recorder gathers the recorded envs' rows after each step, and the day's scenario is decoded
from the device timeline at reset (sng_get_scenario).  Recording synchronises the stream
every step: it is an evaluation / logging tool, not part of the training hot path.

Differences from the reference, by design:
  - values are floats throughout (the reference writes an int 0 where a penalty list was
    empty); numerically identical;
  - for a day started from given arrays (reset_from_initial_values / reset_from_arrays) the
    initial values written are that day's (the reference writes the last *generated* day's, as
    this recorder does for a replayed day);
  - with stochastic PV profiles (pv_noise > 0, not in the reference) 'Available_solar_energy'
    is the noise-free table.
"""
import json
import os

import numpy as np
import torch

from . import _native

RESULT_KEYS = [
    "SOC", "Grid_power", "Grid_energy", "Utilized_solar_energy", "Total_vehicle_penalties",
    "Total_battery_penalties", "Total_penalties", "Available_solar_energy", "Total_cost",
    "Battery_state_of_charge", "Initial_battery_state_of_charge", "Grid_energy_cost", "Battery_action",
    "Charger_actions", "Total_charging_power", "Total_discharging_power", "Charger_power_values",
    "Battery_power_value", "Battery_SOC_below_DoD_penalties", "Low_resource_utilisation_penalties",
    "Battery_overcharging_penalties", "Battery_over_discharging_penalties",
    "Insufficiently_charged_vehicle_penalties", "Needlessly_charged_vehicle_penalties",
    "Overcharged_vehicle_penalties", "Over_discharged_vehicle_penalties", "Battery_calculated_power_value",
    "DisCharging_nonexistent_vehicles_penalties",
]

# smart_nanogrid_environment.py:289-296
FILE_DESTINATIONS = {"training": "training_files", "evaluation": "evaluation_files",
                     "prediction": "single_prediction_files"}


def available_solar_energy(irradiance):
    """PVSystemManager.calculate_available_solar_energy (pv_system_manager.py:67-73, :17)."""
    scaling_pv = 2.279 * 1.134 * 20 * 0.21 / 1000
    return [[float(x * scaling_pv * 1.5) for x in irradiance]]


class DayRecorder:
    """Record the days of envs `env_ids` of a SmartNanogridVecEnv.

    directory=None keeps the records in memory only (`self.last[env]`, and `self.history` when
    keep_history); otherwise every finished day is written as the reference names it, under
    directory/<file destination>/ (one recorded env: the reference's exact file names;
    several: '-env<i>' is inserted before the suffix)."""

    def __init__(self, venv, env_ids=(0,), directory=None, keep_history=False):
        self.venv = venv
        self.env_ids = [int(i) for i in env_ids]
        if not self.env_ids or min(self.env_ids) < 0 or max(self.env_ids) >= venv.num_envs:
            raise ValueError("env_ids must be indices of the batch")
        self.directory = directory
        self.keep_history = keep_history
        self.history = []
        self.last = {}
        self._idx = torch.tensor(self.env_ids, dtype=torch.long, device=venv.device)
        self._steps = {i: [] for i in self.env_ids}
        self._initial = {}
        self._started = False
        venv.attach_recorder(self)
        if venv.timestep == 0:   # attached right after a reset
            self.day_started()

    def close(self):
        self.venv.detach_recorder(self)

    # ------------------------------------------------------------------ hooks (called by the env)
    def day_started(self):
        # a replayed day (reset(generate_new_initial_values=False)) writes the initial values of the last
        # generated day, as the reference's save_initial_values_to_json_file writes
        # generated_initial_values_json (charging_station.py:182-191), which load_initial_values leaves alone
        if not (self.venv._last_reset == "replay" and all(i in self._initial for i in self.env_ids)):
            self._initial = {i: self.venv.get_scenario(i)[0] for i in self.env_ids}
        self._steps = {i: [] for i in self.env_ids}
        self._started = True

    def step_done(self, actions):
        if not self._started:
            return
        v = self.venv
        idx = self._idx
        with torch.cuda.device(v.device):
            scalars = torch.stack([v.info_d[f].index_select(0, idx) for f in _native.INFO_FIELDS]).cpu().numpy()
            power = v.charger_power_d.index_select(0, idx).cpu().numpy()
            soc = v.vehicle_soc_d.index_select(0, idx).cpu().numpy()
            act = actions.index_select(0, idx).cpu().numpy()
        for k, i in enumerate(self.env_ids):
            rec = {f: float(scalars[j, k]) for j, f in enumerate(_native.INFO_FIELDS)}
            rec["charger_power"] = power[k]
            rec["vehicle_soc"] = soc[k]
            rec["actions"] = act[k]
            self._steps[i].append(rec)
        if v.timestep == v.timesteps:
            self._finish_day()

    # ------------------------------------------------------------------ assembly
    def prediction_results(self, env_index):
        """The 28-key dict of the day recorded so far for env `env_index` (reference key order)."""
        v = self.venv
        st = v.settings
        steps = self._steps[env_index]
        N, S, T = st.number_of_chargers, v.slots, v.timesteps
        dt = st.time_interval
        w_b = st.constants.get("battery_penalty_weight", 0.8)
        initial_soc = self._initial[env_index]["SOC"]
        # SOC[c, t] is rewritten by step t (charger.py:37-56); slots no step reached keep their values
        soc = [[float(steps[t]["vehicle_soc"][c]) if t < len(steps) else initial_soc[c][t] for t in range(S)]
               for c in range(N)]
        col = lambda f: [s[f] for s in steps]   # noqa: E731
        zeros = [0.0] * len(steps)
        pen_b, pen_v = col("total_battery_penalty"), col("total_vehicle_penalty")
        if st.pv:
            irr = v.tables()["irr"][:2 * T]
            available = available_solar_energy(irr)
        else:
            available = []
        out = {
            "SOC": soc,
            "Grid_power": col("grid_power"),
            "Grid_energy": [g * dt for g in col("grid_power")],   # central_management_system.py:107
            "Utilized_solar_energy": col("utilized_solar_energy"),
            "Total_vehicle_penalties": pen_v,
            "Total_battery_penalties": pen_b,
            "Total_penalties": [w_b * b + 1 * p for b, p in zip(pen_b, pen_v)],   # penaliser.py:181
            "Available_solar_energy": available,
            "Total_cost": col("total_cost"),
            "Battery_state_of_charge": col("battery_state_of_charge"),
            "Initial_battery_state_of_charge": steps[-1]["initial_battery_soc"] if steps else 0.0,
            "Grid_energy_cost": col("grid_energy_cost"),
            "Battery_action": [float(s["actions"][N]) if st.bess else 0 for s in steps],
            "Charger_actions": [s["actions"][:N].tolist() for s in steps],
            "Total_charging_power": col("total_charging_power"),
            "Total_discharging_power": col("total_discharging_power"),
            "Charger_power_values": [s["charger_power"].tolist() for s in steps],
            "Battery_power_value": col("battery_power_value"),
            "Battery_SOC_below_DoD_penalties": pen_b,                             # penaliser.py:183-184
            "Low_resource_utilisation_penalties": zeros,                          # never computed
            "Battery_overcharging_penalties": zeros,
            "Battery_over_discharging_penalties": zeros,
            "Insufficiently_charged_vehicle_penalties": pen_v,                    # penaliser.py:186-187
            "Needlessly_charged_vehicle_penalties": zeros,
            "Overcharged_vehicle_penalties": zeros,
            "Over_discharged_vehicle_penalties": zeros,
            "Battery_calculated_power_value": col("battery_calculated_power"),
            "DisCharging_nonexistent_vehicles_penalties": col("nonexistent_vehicle_penalty"),
        }
        assert list(out) == RESULT_KEYS
        return out

    def initial_values(self, env_index):
        return self._initial[env_index]

    def file_stem(self, env_index=None):
        """smart_nanogrid_environment.py:300-303"""
        st = self.venv.settings
        name = (f"{st.algorithm_used}-{st.variant_name()}-{st.charging_mode}-{st.penalty_mode_name}-"
                f"{st.number_of_chargers}ch-{st.requested_time_interval}")
        if env_index is not None and len(self.env_ids) > 1:
            name += f"-env{env_index}"
        return name

    def _finish_day(self):
        for i in self.env_ids:
            pr, iv = self.prediction_results(i), self.initial_values(i)
            self.last[i] = (pr, iv)
            if self.keep_history:
                self.history.append((i, pr, iv))
            if self.directory is not None:
                self._write(i, pr, iv)
        self._started = False

    def _write(self, env_index, pr, iv):
        st = self.venv.settings
        path = os.path.join(self.directory, FILE_DESTINATIONS.get(st.environment_mode, ""))
        os.makedirs(path, exist_ok=True)
        stem = os.path.join(path, self.file_stem(env_index))
        with open(stem + "-prediction_results.json", "w") as fp:
            json.dump(pr, fp, indent=4)
        with open(stem + "-initial_values.json", "w") as fp:
            json.dump(iv, fp, indent=4)
