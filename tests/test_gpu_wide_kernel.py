"""GPU: the step kernel BASELINE config 5's bench times -- `void sng::step_wide_kernel<50, L, true, false, true>`
(N = 50, 15-minute steps, extended day, stochastic PV / price profiles, packed device-RNG day records,
no diagnostics) -- pinned to the CPU oracle.

Device-RNG days are exported in the reference's initial_values layout (sng_get_scenario) and loaded into
oracle envs seeded like the GPU's envs (global env i <- seed + i), so the oracle draws the same day's
profile factors (the day counter advances once per loaded day on both sides).  Both are stepped with
Box-uniform actions (chargers U[0, 1], BESS U[-1, 1], 20 % exact zeros, 5 % exact upper bounds, a quarter
of the envs discharging the BESS at -1 most steps), two consecutive days, bit-exact on the sampled envs
(the oracle squares with x*x here, as the GPU does).  The full population runs against the general
(diagnostics) kernel on the same days and actions, bit-exact on every env.
"""
import ctypes

import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smart_nanogrid_gym import SmartNanogridVecEnv  # noqa: E402
from test_gpu_bench_kernel import actions, load_day  # noqa: E402

CONFIG5 = dict(number_of_chargers=50, time_interval="15min", charging_mode="bounded",
               vehicle_uncharged_penalty_mode="sparse", pv_system_available_in_model=True,
               battery_system_available_in_model=True, extended_day=True, pv_noise=0.2, price_noise=0.1)
WIDE_KERNEL = ("void sng::step_wide_kernel<50, ", ", true, false, true>")   # <N, lanes, PK, REQ, NOISE>


@pytest.fixture(scope="module", autouse=True)
def _square_mode():
    O.lib().orc_set_square_mode.argtypes = [ctypes.c_int]
    O.lib().orc_set_square_mode(1)
    yield
    O.lib().orc_set_square_mode(0)


@pytest.mark.parametrize("E,sample", [(4096, 256), (65536, 128)])
def test_wide_step_kernel_device_days_vs_oracle_and_general(E, sample):
    seed = 77
    venv = SmartNanogridVecEnv(E, seed=seed, rng="device", **CONFIG5)
    diag = SmartNanogridVecEnv(E, seed=seed, rng="device", info=True, **CONFIG5)
    ids = np.sort(np.random.default_rng(3).choice(E, sample, replace=False))
    cfg = O.OracleConfig(**CONFIG5)
    envs = [O.OracleEnv(cfg, seed + int(i)) for i in ids]
    rng = np.random.default_rng(E)
    heavy = (np.arange(E) % 4) == 0
    saw = dict(clamp=0, dod=0)
    for day in range(2):
        obs = venv.reset_tensors().cpu().numpy()
        name = venv.step_kernel_name()
        assert name.startswith(WIDE_KERNEL[0]) and name.endswith(WIDE_KERNEL[1]), name
        np.testing.assert_array_equal(obs, diag.reset_tensors().cpu().numpy())
        days = [venv.get_scenario(int(i)) for i in ids]   # the sampled envs' days only
        ref0 = np.stack([load_day(e, iv, ratio) for e, (iv, ratio) in zip(envs, days)])
        np.testing.assert_array_equal(obs[ids], ref0, err_msg=f"day {day} reset")
        for t in range(venv.timesteps):
            a = actions(rng, E, 51, heavy)
            ad = torch.from_numpy(a).to(venv.device)
            o, r, d = venv.step_tensors(ad)
            od, rd, _ = diag.step_tensors(ad)
            o, r = o.cpu().numpy(), r.cpu().numpy()
            np.testing.assert_array_equal(o, od.cpu().numpy(), err_msg=f"day {day} t {t}: vs general kernel")
            np.testing.assert_array_equal(r, rd.cpu().numpy(), err_msg=f"day {day} t {t}: vs general kernel")
            outs = [e.step(a[i]) for e, i in zip(envs, ids)]
            np.testing.assert_array_equal(o[ids], np.stack([x[0] for x in outs]), err_msg=f"day {day} t {t}")
            np.testing.assert_array_equal(r[ids], np.array([x[1] for x in outs]))
            assert bool(d.cpu().numpy().all()) == (t == venv.timesteps - 1)
            infos = [x[3] for x in outs]
            saw["clamp"] += sum(1 for inf in infos if inf["bess_power"] < 0 and inf["bess_soc"] == 0.0)
            saw["dod"] += sum(1 for inf in infos if inf["pen_battery"] > 0)
        np.testing.assert_array_equal(venv.battery_state_of_charge()[ids], np.array([e.bess_soc for e in envs]))
        np.testing.assert_array_equal(venv.return_d.cpu().numpy(), diag.return_d.cpu().numpy())
    assert saw["clamp"] > 0 and saw["dod"] > 0, saw
    venv.close()
    diag.close()


# every N = 50 station without diagnostics steps through the wide kernel, not only config 5.  A V2X
# station (negative charger actions: the wave-uniform rolled path, numpy's pairwise order over both signs and
# the inverted discharge flag, charger.py:108-140) and a station without BESS (act_dim = N, no BESS tail) on
# 1 h device days, against the oracle on sampled envs and the general kernel on every env.
WIDE_VARIANTS = {
    "v2x": dict(number_of_chargers=50, time_interval="1h", charging_mode="bounded",
                vehicle_uncharged_penalty_mode="dense", pv_system_available_in_model=True,
                battery_system_available_in_model=True, vehicle_to_everything=True),
    "no_bess": dict(number_of_chargers=50, time_interval="1h", charging_mode="bounded",
                    vehicle_uncharged_penalty_mode="on_departure", pv_system_available_in_model=True,
                    battery_system_available_in_model=False),
}


@pytest.mark.parametrize("variant", sorted(WIDE_VARIANTS))
def test_wide_step_kernel_other_stations_vs_oracle(variant):
    kw = WIDE_VARIANTS[variant]
    E, sample, seed = 4096, 192, 31
    venv = SmartNanogridVecEnv(E, seed=seed, rng="device", **kw)
    diag = SmartNanogridVecEnv(E, seed=seed, rng="device", info=True, **kw)
    ids = np.sort(np.random.default_rng(5).choice(E, sample, replace=False))
    cfg = O.OracleConfig(**kw)
    envs = [O.OracleEnv(cfg, 0) for _ in ids]   # the days come from the GPU
    rng = np.random.default_rng(11)
    lo, hi = venv.action_space.low, venv.action_space.high
    A = venv.act_dim
    saw_neg = 0
    for day in range(2):
        obs = venv.reset_tensors().cpu().numpy()
        name = venv.step_kernel_name()
        assert name.startswith("void sng::step_wide_kernel<50, "), name
        np.testing.assert_array_equal(obs, diag.reset_tensors().cpu().numpy())
        ivs, ratios = venv.get_scenarios(0, E)
        ref0 = np.stack([load_day(e, ivs[i], ratios[i]) for e, i in zip(envs, ids)])
        np.testing.assert_array_equal(obs[ids], ref0, err_msg=f"{variant} day {day} reset")
        for t in range(venv.timesteps):
            a = (lo + (hi - lo) * rng.random((E, A))).astype(np.float32)
            r = rng.random(a.shape)
            a[r < 0.2] = 0.0
            a[(r >= 0.2) & (r < 0.25)] = hi[np.nonzero((r >= 0.2) & (r < 0.25))[1]]
            ad = torch.from_numpy(a).to(venv.device)
            o, rw, d = venv.step_tensors(ad)
            od, rd, _ = diag.step_tensors(ad)
            o, rw = o.cpu().numpy(), rw.cpu().numpy()
            np.testing.assert_array_equal(o, od.cpu().numpy(), err_msg=f"{variant} day {day} t {t}: vs general")
            np.testing.assert_array_equal(rw, rd.cpu().numpy(), err_msg=f"{variant} day {day} t {t}: vs general")
            outs = [e.step(a[i]) for e, i in zip(envs, ids)]
            np.testing.assert_array_equal(o[ids], np.stack([x[0] for x in outs]), err_msg=f"{variant} d{day} t{t}")
            np.testing.assert_array_equal(rw[ids], np.array([x[1] for x in outs]))
            assert bool(d.cpu().numpy().all()) == (t == venv.timesteps - 1)
            saw_neg += int((a[ids, :50] < 0).sum())
    assert (saw_neg > 0) == (variant == "v2x")
    venv.close()
    diag.close()
