"""Helpers to read the golden fixtures written by tests/golden/make_golden.py."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = os.path.join(GOLDEN, "kat")


def cases():
    with open(os.path.join(GOLDEN, "cases.json")) as fp:
        return json.load(fp)


def case(name):
    meta = [m for m in cases() if m["name"] == name][0]
    return meta, np.load(os.path.join(GOLDEN, f"{name}.npz"))


def eval_cases():
    """The solvers/evaluator.py:88-101 replay cases (make_golden.py run_evaluator_case)."""
    with open(os.path.join(GOLDEN, "eval_cases.json")) as fp:
        return json.load(fp)


def eval_case(name):
    meta = [m for m in eval_cases() if m["name"] == name][0]
    return meta, np.load(os.path.join(GOLDEN, f"{name}.npz"))


def load_case(meta):
    return np.load(os.path.join(GOLDEN, f"{meta['name']}.npz"))


def kat(sub):
    """Recorded PPO episode (reference solvers/RL/<sub>/PPO-b-pv-bounded-sparse-4ch-1h-*.json)."""
    with open(os.path.join(KAT, f"{sub}-initial_values.json")) as fp:
        iv = json.load(fp)
    with open(os.path.join(KAT, f"{sub}-prediction_results.json")) as fp:
        pr = json.load(fp)
    N = len(iv["SOC"])
    V = max(len(a) for a in iv["Arrivals"])
    arr = np.full((N, V), -1, np.int64)
    dep = np.full((N, V), -1, np.int64)
    for c in range(N):
        arr[c, :len(iv["Arrivals"][c])] = iv["Arrivals"][c]
        dep[c, :len(iv["Departures"][c])] = iv["Departures"][c]
    av = np.array(pr["Available_solar_energy"][0])
    us = np.array(pr["Utilized_solar_energy"])
    k = int(np.argmax(av[:24]))
    ratio = round(us[k] / av[k] * 100) / 100   # ratio = randint(0,180)/100, recovered from the record
    actions = np.array([pr["Charger_actions"][t] + [pr["Battery_action"][t]] for t in range(24)], np.float32)
    return dict(N=N, iv=iv, pr=pr, arrivals=arr, departures=dep, ratio=ratio, actions=actions,
                bess_soc0=pr["Initial_battery_state_of_charge"])
