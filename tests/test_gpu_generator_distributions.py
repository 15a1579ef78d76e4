"""GPU: the device-RNG day generator (generate_kernel) against the reference's vehicle process.

Device days are drawn from counter-based hash streams, not from numpy's MT19937, so their parity with
the reference is distributional.  Days are exported through get_scenarios (the
reference's initial_values layout) and each vehicle read back as (arrival step, departure step, capacity,
arrival SoC, requested SoC).  Against the law of ChargingStation.generate_initial_vehicle_presence_per_
charger (charging_station.py:200-279):
  - capacity ~ U{15..119} (randint(15, 120), :267-269): chi-square goodness of fit;
  - arrival SoC ~ U(0.1, 0.9) (:257-259): Kolmogorov-Smirnov (the device draws it as a float32 value);
  - requested SoC ~ U(soc + 0.1, 1) (:261-265): KS of (req - soc - 0.1) / (0.9 - soc) against U(0, 1);
and against oracle days (the C restatement, pinned draw for draw to the reference's generator), same
configuration: the histograms of arrivals per charger-day (at 1 h at most 5, mean ~3.02 -- SURVEY.md
section 8a R3), of stay lengths (departure - arrival) and of arrival steps, by chi-square tests of
homogeneity.  Stations of 10 and 50 chargers, 1 h and 15-minute (extended) days.  Seeds are fixed, so
the outcome is deterministic; the p-value floor 1e-4 is what a correct generator passes at these sample
sizes and a biased one (a wrong arrival probability, departure window or capacity range) fails by many
orders of magnitude.
"""
import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")
stats = pytest.importorskip("scipy.stats")
pytestmark = pytest.mark.gpu

from smart_nanogrid_gym import SmartNanogridVecEnv  # noqa: E402

P_MIN = 1e-4


def _vehicles_device(venv, days):
    """Per vehicle (arrival, departure, capacity, SoC, requested SoC) and arrivals per charger-day."""
    veh, per_day = [], []
    for _ in range(days):
        venv.reset_tensors()
        ivs, _ = venv.get_scenarios()
        for d in ivs:
            for c, arrs in enumerate(d["Arrivals"]):
                per_day.append(len(arrs))
                for a, dep in zip(arrs, d["Departures"][c]):
                    veh.append((a, dep, d["Vehicle_capacities"][c][a], d["SOC"][c][a], d["Requested_SOC"][c][a]))
        for t in range(venv.timesteps):   # step through the day so the next reset draws a new one
            venv.step_tensors(torch.zeros((venv.num_envs, venv.act_dim), device=venv.device))
    return np.array(veh, np.float64), np.array(per_day)


def _vehicles_oracle(kw, envs, seed0):
    cfg = O.OracleConfig(**kw)
    veh, per_day = [], []
    for i in range(envs):
        e = O.OracleEnv(cfg, seed0 + i)
        e.reset()
        sc = e.scenario()
        for c in range(cfg.N):
            arrs = sc["arrivals"][c][sc["arrivals"][c] >= 0]
            deps = sc["departures"][c][sc["departures"][c] >= 0]
            per_day.append(len(arrs))
            for a, dep in zip(arrs, deps):
                veh.append((a, dep, sc["cap"][c][a], sc["soc"][c][a], sc["req"][c][a]))
    return np.array(veh, np.float64), np.array(per_day)


def _homogeneous(x, y, name):
    """Chi-square test of homogeneity of two integer samples, sparse tail bins merged."""
    lo, hi = int(min(x.min(), y.min())), int(max(x.max(), y.max()))
    cx = np.bincount((x - lo).astype(int), minlength=hi - lo + 1).astype(float)
    cy = np.bincount((y - lo).astype(int), minlength=hi - lo + 1).astype(float)
    table, acc = [], np.zeros(2)
    for a, b in zip(cx, cy):   # merge adjacent bins until each merged bin holds >= 20 of both samples
        acc += (a, b)
        if acc.min() >= 20:
            table.append(acc.copy())
            acc[:] = 0
    if acc.sum() > 0:
        table[-1] += acc
    p = stats.chi2_contingency(np.array(table).T)[1]
    assert p > P_MIN, f"{name}: device and reference histograms differ (p = {p:.2e})"
    return p


@pytest.mark.parametrize("N,interval,E,days,ref_envs", [(10, "1h", 4096, 2, 3000), (50, "1h", 1024, 2, 600),
                                                        (10, "15min", 2048, 2, 2000), (50, "15min", 512, 2, 500)])
def test_device_generator_distributions(N, interval, E, days, ref_envs):
    kw = dict(number_of_chargers=N, time_interval=interval, charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse", enable_requested_state_of_charge=True)
    if interval != "1h":
        kw["extended_day"] = True
    venv = SmartNanogridVecEnv(E, seed=31 + N, rng="device", **kw)
    T = venv.timesteps
    dev, dev_n = _vehicles_device(venv, days)
    venv.close()
    ref, ref_n = _vehicles_oracle(kw, ref_envs, 70_000 + N)
    arr, dep, cap, soc, req = dev.T

    # the reference's per-vehicle laws, directly
    p_cap = stats.chisquare(np.bincount(cap.astype(int) - 15, minlength=105)[:105])[1]
    assert cap.min() >= 15 and cap.max() <= 119 and p_cap > P_MIN, p_cap
    p_soc = stats.kstest(soc, "uniform", args=(0.1, 0.8))[1]
    assert soc.min() >= 0.1 and soc.max() <= 0.9 and p_soc > P_MIN, p_soc
    u = (req - soc - 0.1) / (0.9 - soc)
    p_req = stats.kstest(u, "uniform")[1]
    assert u.min() >= 0.0 and u.max() <= 1.0 and p_req > P_MIN, p_req

    # the process, against the reference generator's days
    if interval == "1h":
        assert dev_n.max() <= 5 and abs(dev_n.mean() - 3.02) < 0.05, (dev_n.max(), dev_n.mean())
    assert abs(dev_n.mean() - ref_n.mean()) < 4 * np.hypot(dev_n.std() / np.sqrt(dev_n.size),
                                                            ref_n.std() / np.sqrt(ref_n.size)) + 1e-9
    _homogeneous(dev_n, ref_n, "arrivals per charger-day")
    _homogeneous(dep - arr, ref[:, 1] - ref[:, 0], "stay length")
    _homogeneous(arr, ref[:, 0], "arrival step")
    assert arr.min() >= 0 and arr.max() < T


@pytest.mark.parametrize("N", [10, 50])
def test_arrival_soc_codes(N):
    """Device days carry the arrival SoC in their 2 B records as a 13-bit code (sng_layout.h code_soc): every
    exported arrival SoC is one of the 8,192 float32 values 0.1f + 0.8f (k + 0.5) / 8192 and the draws cover that
    grid evenly (the KS test above checks the law).  Round 5 measured 4 B records carrying any float32 value on
    the headline station: 0.15-0.18 us more per step (profiles/r05_ab_records_4b.txt), so the grid stays."""
    kw = dict(number_of_chargers=N, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    v = SmartNanogridVecEnv(4096, seed=77, rng="device", **kw)
    veh, _ = _vehicles_device(v, 2)
    v.close()
    soc = veh[:, 3]
    assert soc.size > 20000 and np.all(soc == soc.astype(np.float32))
    k = np.arange(8192, dtype=np.float32)
    grid = np.float32(0.1) + np.float32(0.8) * ((k + np.float32(0.5)) * np.float32(1.0 / 8192.0))
    assert np.isin(soc.astype(np.float32), grid).all()
    counts = np.bincount(np.searchsorted(grid, soc.astype(np.float32)), minlength=8192)
    assert stats.chisquare(counts).pvalue > P_MIN
