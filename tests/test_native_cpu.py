"""CPU-side checks of the product library (no GPU calls): the C ABI loads and exports every
symbol include/sng.h declares, and the host reference-RNG day generator reproduces the
reference's days (golden vectors) and the oracle's days draw for draw."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as O
from golden_util import case, cases
from smart_nanogrid_gym import EnvSettings, _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "sng.h")).read()
    return sorted(set(re.findall(r"\b(sng_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_native.EXPORTS), "ctypes binding out of sync with include/sng.h"
    assert L.sng_abi_version() == 10


def test_config_defaults_are_reference_constants():
    cfg = _native.SngConfig()
    _native.lib().sng_config_defaults(ctypes.byref(cfg))
    assert cfg.number_of_chargers == 8 and cfg.time_interval_hours == 1.0
    assert (cfg.bess_capacity_kwh, cfg.bess_initial_soc, cfg.bess_max_charging_kw) == (80, 0.5, 44)
    assert (cfg.bess_charging_efficiency, cfg.bess_depth_of_discharge) == (0.95, 0.15)
    assert (cfg.ev_max_power_kw, cfg.ev_efficiency) == (22, 0.95)
    assert (cfg.grid_cost_weight, cfg.battery_penalty_weight, cfg.selling_price_coefficient) == (0.75, 0.8, 0.8)


def test_create_rejects_configs_the_reference_cannot_run():
    L = _native.lib()
    for kw in [dict(time_interval="15min"), dict(number_of_chargers=0), dict(number_of_chargers=129)]:
        cfg = EnvSettings(charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse", **kw).to_native()
        h = ctypes.c_void_p()
        rc = L.sng_create(ctypes.byref(cfg), 0, 4, 0, ctypes.byref(h))
        assert rc != 0 and not h.value
        assert L.sng_last_error(None)


def test_settings_errors_match_reference():
    with pytest.raises(ValueError, match="Wrong time interval"):
        EnvSettings(time_interval="3d")
    with pytest.raises(TypeError):
        EnvSettings(price_model=5)


def host_days(kwargs, n_envs, seed, episodes, V=8):
    s = EnvSettings(**kwargs)
    cfg = s.to_native()
    N = s.number_of_chargers
    S = s.timesteps + 1 if kwargs.get("extended_day") else 25
    shp = (episodes, n_envs, N, S)
    soc, occ, cap, req = (np.zeros(shp) for _ in range(4))
    arr = np.zeros((episodes, n_envs, N, V), np.int32)
    dep = np.zeros((episodes, n_envs, N, V), np.int32)
    ratio = np.zeros((episodes, n_envs))
    P, I = _native.c_double_p, _native.c_int32_p
    rc = _native.lib().sng_host_generate_scenarios(
        ctypes.byref(cfg), n_envs, seed, episodes, soc.ctypes.data_as(P), occ.ctypes.data_as(P),
        cap.ctypes.data_as(P), req.ctypes.data_as(P), arr.ctypes.data_as(I), dep.ctypes.data_as(I), V,
        ratio.ctypes.data_as(P))
    assert rc == 0
    return dict(soc=soc, occ=occ, cap=cap, req=req, arrivals=arr, departures=dep, ratio=ratio)


@pytest.mark.parametrize("name", [m["name"] for m in cases()])
def test_host_generator_reproduces_reference_days(name):
    meta, d = case(name)
    days = host_days(meta["kwargs"], 1, meta["seed"], meta["n_episodes"])
    for ep in range(meta["n_episodes"]):
        for k, g in [("soc", "soc0"), ("occ", "occ"), ("cap", "cap"), ("req", "req"), ("arrivals", "arrivals"),
                     ("departures", "departures")]:
            np.testing.assert_array_equal(days[k][ep, 0], d[g][ep], err_msg=f"{k} ep{ep}")
        assert days["ratio"][ep, 0] == d["ratio"][ep]


def test_host_generator_matches_oracle_many_seeds():
    kw = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse", enable_requested_state_of_charge=True)
    E, seed = 200, 777
    days = host_days(kw, E, seed, 2)
    cfg = O.OracleConfig(**kw)
    for i in range(0, E, 7):
        env = O.OracleEnv(cfg, seed + i)
        for ep in range(2):
            env.reset()
            sc = env.scenario()
            for k in ["soc", "occ", "cap", "req", "arrivals", "departures"]:
                np.testing.assert_array_equal(days[k][ep, i], sc[k])
            assert days["ratio"][ep, i] == env.ratio
            for t in range(cfg.T):   # advance the oracle through the day (consumes the day-end draw)
                env.step(np.zeros(cfg.act_dim, np.float32))


CONFIG5 = dict(number_of_chargers=50, time_interval="15min", charging_mode="bounded",
               vehicle_uncharged_penalty_mode="sparse", extended_day=True, pv_noise=0.2, price_noise=0.1)


def test_extended_day_host_generator_matches_oracle():
    """Build-defined extended day (N=50, 15 min, T=96, T+1 slots): the
    library's host generator and the oracle draw the same days from the reference's streams."""
    E, seed = 24, 4242
    days = host_days(CONFIG5, E, seed, 2)
    assert days["soc"].shape[-1] == 97
    cfg = O.OracleConfig(**CONFIG5)
    assert cfg.T == 96 and cfg.slots == 97
    for i in range(0, E, 5):
        env = O.OracleEnv(cfg, seed + i)
        for ep in range(2):
            env.reset()
            sc = env.scenario(vmax=8)
            for k in ["soc", "occ", "cap", "req", "arrivals", "departures"]:
                np.testing.assert_array_equal(days[k][ep, i], sc[k])
            assert days["ratio"][ep, i] == env.ratio
            for t in range(cfg.T):
                env.step(np.zeros(cfg.act_dim, np.float32))


def test_extended_day_tables_and_profiles():
    cfg = O.OracleConfig(**CONFIG5)
    tb = cfg.tables()
    assert tb["price"].size == 192 and tb["irr"].size == 192
    low, high = tb["price"].min(), tb["price"].max()
    # per-step tariff loop (accountant.py:61-68): low for i < 7/dt or i > 19/dt
    for i in range(96):
        assert tb["price"][i] == (low if (i < 28 or i > 76) else high)
        assert tb["price"][i + 96] == tb["price"][i]
    env = O.OracleEnv(cfg, 5)
    env.reset()
    f1 = env.profiles()
    env.reset()
    f2 = env.profiles()
    for (pv, pr), (pv2, pr2) in [(f1, f2)]:
        assert pv.size == 99 and np.all(np.abs(pv - 1) <= 0.2) and np.all(np.abs(pr - 1) <= 0.1)
        assert not np.array_equal(pv, pv2)   # a new day draws new profiles
    # standard configs keep the reference's 25 slots and refuse T > 24
    with pytest.raises(IndexError):
        O.OracleEnv(O.OracleConfig(number_of_chargers=2, time_interval="15min"), 0)


def test_create_rejects_extended_day_without_flag():
    kw = dict(CONFIG5)
    kw.pop("extended_day")
    s = EnvSettings(**kw)
    cfg = s.to_native()
    h = ctypes.c_void_p()
    rc = _native.lib().sng_create(ctypes.byref(cfg), 0, 4, 0, ctypes.byref(h))
    assert rc != 0 and b"extended_day" in _native.lib().sng_last_error(None)


def test_python_constants_mirror_the_header():
    """The flag bits and the flag-summary word count of include/sng.h, as the Python layer uses them."""
    import re
    text = open(os.path.join(ROOT, "include", "sng.h")).read()
    defs = {k: int(v, 0) for k, v in re.findall(r"#define SNG_(FLAG_\w+)\s+(0x[0-9a-fA-F]+|\d+)u?", text)}
    assert defs["FLAG_SUMMARY_WORDS"] == _native.FLAG_SUMMARY_WORDS
    for k in ("FLAG_NEGATIVE_DEMAND", "FLAG_CHARGING_MODE", "FLAG_BESS_SOC_ABOVE_1", "FLAG_V2X_BREAKPOINT"):
        assert defs[k] == getattr(_native, k), k
