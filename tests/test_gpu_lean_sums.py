"""GPU: the lean step kernel's charging / discharging totals (csrc/sng_kernels.hip, step_lean).

The lean step (N <= 16, one lane per env, no diagnostics, NumPy-2 promotion, power-of-two dt) keeps the
running sums of the positive and negative charger powers and uses them as numpy's pairwise sums of the
compacted arrays (charging_station.py:289-293) whenever that is provably exact; other lanes compact their
powers into LDS and run the pairwise sum.  These tests drive both branches on purpose -- tiny and
subnormal charging actions (8+ positive float32 powers whose sum is not exact), near-full discharges at
V2X stations (8+ negative powers), ordinary Box actions -- and require:
  - the lean kernel's observations and rewards bit-exact against the general (diagnostics) kernel on the
    same days and actions, for every env, and against the CPU oracle for a sample of envs;
  - the slow branch to have been needed, and to have mattered (the running sum differs from numpy's
    pairwise sum) in some env-steps, judged from the per-charger powers the diagnostics kernel reports.
"""
import ctypes

import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smart_nanogrid_gym import SmartNanogridVecEnv  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _square_mode():
    O.lib().orc_set_square_mode.argtypes = [ctypes.c_int]
    O.lib().orc_set_square_mode(1)
    yield
    O.lib().orc_set_square_mode(0)


def _actions(rng, E, N, v2x):
    """Per env category (env % 4): Box-uniform; tiny positive (10^U(-12, 0)); heavy discharge (V2X) or
    near-full charge; a mix of subnormal, tiny and full-scale values.  20 % exact zeros throughout."""
    a = np.empty((E, N + 1), np.float32)
    lo = -1.0 if v2x else 0.0
    cat = np.arange(E) % 4
    a[:, :N] = rng.uniform(lo, 1.0, (E, N))
    m = cat == 1
    a[m, :N] = 10.0 ** rng.uniform(-12, 0, (m.sum(), N))
    m = cat == 2
    a[m, :N] = (-1.0 if v2x else 1.0) * rng.uniform(0.6, 1.0, (m.sum(), N))
    m = cat == 3
    a[m, :N] = rng.choice(np.array([1e-40, 1e-30, 3e-8, 1.0, 0.5, -0.0], np.float32), (m.sum(), N))
    a[:, N] = rng.uniform(-1.0, 1.0, E)
    a[rng.random(a.shape) < 0.2] = 0.0
    return a


def _seq(x):
    s = 0.0
    for v in x:
        s += v
    return s


@pytest.mark.parametrize("N,v2x", [(10, True), (16, True), (8, True), (10, False), (16, False), (50, True), (50, False)])
def test_lean_totals_vs_general_kernel_and_oracle(N, v2x):
    """N = 50 is BASELINE config 5's station (15-minute steps, extended day, stochastic profiles), stepped by
    the wide lean kernel: running sums where exact, the positive powers rebuilt from the records and the
    actions where not, and a wavefront with a discharging action in numpy's order throughout."""
    E, seed = 2048, 4242 + N
    kw = dict(number_of_chargers=N, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse", pv_system_available_in_model=True,
              battery_system_available_in_model=True, vehicle_to_everything=v2x)
    if N == 50:
        kw.update(time_interval="15min", extended_day=True, pv_noise=0.2, price_noise=0.1)
    lean = SmartNanogridVecEnv(E, seed=seed, rng="reference", **kw)
    lean._info.flags = None
    diag = SmartNanogridVecEnv(E, seed=seed, rng="reference", info=True, **kw)
    diag._enable_info(per_charger=True)
    name = lean.step_kernel_name()
    if N == 50:
        assert name.startswith("void sng::step_wide_kernel<50, ") and name.endswith(", false, false, true>"), name
    elif N == 10 and not v2x:   # the headline station steps through the wide kernel (two lanes per env)
        assert name.startswith("void sng::step_wide_kernel<10, ") and name.endswith(", false, false, false>"), name
    else:
        assert name == f"void sng::step_lean_kernel<{N}, false, false>"
    T = lean.timesteps
    ids = np.arange(0, E, 16)
    cfg = O.OracleConfig(**kw)
    envs = [O.OracleEnv(cfg, seed + int(i)) for i in ids]
    rng = np.random.default_rng(N)
    need_pos = need_neg = mattered = 0
    for day in range(2):
        o_l = lean.reset_tensors().cpu().numpy()
        o_d = diag.reset_tensors().cpu().numpy()
        np.testing.assert_array_equal(o_l, o_d)
        np.testing.assert_array_equal(o_l[ids], np.stack([e.reset() for e in envs]))
        for t in range(T):
            a = _actions(rng, E, N, v2x)
            ad = torch.from_numpy(a).to(lean.device)
            ol, rl, _ = lean.step_tensors(ad)
            od, rd, _ = diag.step_tensors(ad)
            ol, rl, od, rd = ol.cpu().numpy(), rl.cpu().numpy(), od.cpu().numpy(), rd.cpu().numpy()
            np.testing.assert_array_equal(ol, od, err_msg=f"day {day} t {t}: obs, lean vs general")
            np.testing.assert_array_equal(rl, rd, err_msg=f"day {day} t {t}: reward, lean vs general")
            outs = [e.step(a[i]) for e, i in zip(envs, ids)]
            np.testing.assert_array_equal(ol[ids], np.stack([x[0] for x in outs]), err_msg=f"day {day} t {t}")
            np.testing.assert_array_equal(rl[ids], np.array([x[1] for x in outs]))
            pw = diag.charger_power_d.cpu().numpy()
            for row in pw:
                pos, neg = row[row > 0], row[row < 0]
                if len(neg) >= 8:
                    need_neg += 1
                    mattered += _seq(neg) != O.pairwise_sum(neg)
                if len(pos) >= 8 and not (_seq(pos) <= pos.min() * 2.0 ** 28):
                    need_pos += 1
                    mattered += _seq(pos) != O.pairwise_sum(pos)
    # the slow branch was needed for positives (and for negatives at V2X stations), and it mattered
    assert need_pos > 0 and mattered > 0, (need_pos, need_neg, mattered)
    if v2x:
        assert need_neg > 0, need_neg
    lean.close()
    diag.close()
