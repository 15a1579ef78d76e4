"""GPU: the step kernel the headline bench times -- `void sng::step_wide_kernel<10, 2, true, false, false>`
(N = 10, two lanes per env, 32 envs per wavefront, no diagnostics, NumPy-2 / power-of-two dt fast path, packed device-RNG day
records) -- pinned directly to the CPU oracle.

Device-RNG days (GPU generator, as in the bench) are exported in the reference's initial_values layout
(sng_get_scenario), loaded into oracle envs with the same PV ratio, and both are stepped with the same
Box-uniform actions: chargers U[0, 1], BESS U[-1, 1] (negative actions included), 20 % exact zeros, 5 %
exactly the upper bound, and a quarter of the envs discharging the BESS at -1 most steps (the
over-discharge clamp and the DoD penalty, battery_energy_storage_system.py:76-106, penaliser.py:104-111).
Observations and rewards must be bit-exact (the oracle squares with x*x here, as the GPU does).
Two consecutive days, so the BESS state carried across the reset is checked too.
"""
import ctypes

import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smart_nanogrid_gym import SmartNanogridVecEnv  # noqa: E402

# the headline's step kernel: the wide kernel with two lanes per env
BENCH_KERNELS = ("void sng::step_wide_kernel<10, 2, true, false, false>",)
KW = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse",
          pv_system_available_in_model=True, battery_system_available_in_model=True)


@pytest.fixture(scope="module", autouse=True)
def _square_mode():
    O.lib().orc_set_square_mode.argtypes = [ctypes.c_int]
    O.lib().orc_set_square_mode(1)
    yield
    O.lib().orc_set_square_mode(0)


def load_day(env, iv, ratio, V=8):
    N = len(iv["SOC"])
    arr = np.full((N, V), -1, np.int32)
    dep = np.full((N, V), -1, np.int32)
    for c in range(N):
        arr[c, :len(iv["Arrivals"][c])] = iv["Arrivals"][c]
        dep[c, :len(iv["Departures"][c])] = iv["Departures"][c]
    return env.load(iv["SOC"], iv["Charger_occupancy"], iv["Vehicle_capacities"], iv["Requested_SOC"], arr, dep, ratio)


def actions(rng, E, A, heavy):
    a = np.empty((E, A), np.float32)
    a[:, :A - 1] = rng.uniform(0.0, 1.0, (E, A - 1))
    a[:, A - 1] = rng.uniform(-1.0, 1.0, E)
    r = rng.random(a.shape)
    a[r < 0.2] = 0.0
    a[(r >= 0.2) & (r < 0.25)] = 1.0
    a[heavy & (rng.random(E) < 0.7), A - 1] = -1.0
    return a


@pytest.mark.parametrize("E,sample", [(4096, None), (65536, 512)])
def test_benched_step_kernel_vs_oracle(E, sample):
    venv = SmartNanogridVecEnv(E, seed=2024, rng="device", **KW)   # info=False: the bench's variant
    venv._info.flags = None                                        # the bench passes no flag array either
    ids = np.arange(E) if sample is None else np.sort(np.random.default_rng(9).choice(E, sample, replace=False))
    cfg = O.OracleConfig(**KW)
    envs = [O.OracleEnv(cfg, 0) for _ in ids]   # the days come from the GPU: the oracle's own RNG is unused
    rng = np.random.default_rng(E)
    heavy = (np.arange(E) % 4) == 0
    saw = dict(neg_bess=0, clamp=0, dod=0)
    for day in range(2):
        obs = venv.reset_tensors().cpu().numpy()
        assert venv.step_kernel_name() in BENCH_KERNELS
        ivs, ratios = venv.get_scenarios(0, E)
        ref0 = np.stack([load_day(e, ivs[i], ratios[i]) for e, i in zip(envs, ids)])
        np.testing.assert_array_equal(obs[ids], ref0, err_msg=f"day {day} reset")
        for t in range(24):
            a = actions(rng, E, 11, heavy)
            o, r, d = venv.step_tensors(torch.from_numpy(a).to(venv.device))
            outs = [e.step(a[i]) for e, i in zip(envs, ids)]
            np.testing.assert_array_equal(o.cpu().numpy()[ids], np.stack([x[0] for x in outs]),
                                          err_msg=f"day {day} t {t}")
            np.testing.assert_array_equal(r.cpu().numpy()[ids], np.array([x[1] for x in outs]))
            assert bool(d.cpu().numpy().all()) == (t == 23)
            infos = [x[3] for x in outs]
            saw["neg_bess"] += int((a[ids, -1] < 0).sum())
            saw["clamp"] += sum(1 for inf in infos if inf["bess_power"] < 0 and inf["bess_soc"] == 0.0)
            saw["dod"] += sum(1 for inf in infos if inf["pen_battery"] > 0)
        np.testing.assert_array_equal(venv.battery_state_of_charge()[ids], np.array([e.bess_soc for e in envs]))
    # the discharge branch, its over-discharge clamp and the DoD penalty were all exercised
    assert saw["neg_bess"] > 0 and saw["clamp"] > 0 and saw["dod"] > 0, saw
    venv.close()
