"""GPU: the SB3 VecEnv contract and the C ABI's state getters.

* seed() reseeds: after venv.seed(s) the next days are those of a fresh population seeded s (both RNG
  modes; SB3 VecEnv.seed semantics, env i <- s + i).
* get_attr / set_attr / env_method honour `indices` env by env, and raise for unknown names or for
  batch-wide settings set on a subset.
* ABI getters report argument errors through sng_last_error and synchronise only the caller's stream.
* Device-RNG days of wide stations (N > 16: the generator without its fused t = 0 blocks) draw their PV
  ratio and zero the t = 0 penalty like the fused path, and every device day advances the day counter
  exactly once.
* A steps-only graph refuses a day of another encoding and a start after t = 0.
"""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv  # noqa: E402
from smart_nanogrid_gym import _native  # noqa: E402
from smart_nanogrid_gym._native import NativeError, lib  # noqa: E402

KW = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")


@pytest.mark.parametrize("rng", ["reference", "device"])
def test_seed_reseeds_the_streams(rng):
    E = 512
    a = SmartNanogridVecEnv(E, seed=1, rng=rng, **KW)
    a.reset_tensors()
    for t in range(24):
        a.step_tensors(torch.zeros((E, 11), device="cuda:0"))
    assert a.seed(77) == [77 + i for i in range(E)]
    b = SmartNanogridVecEnv(E, seed=77, rng=rng, **KW)
    for day in range(2):
        oa, ob = a.reset_tensors().clone(), b.reset_tensors().clone()
        assert torch.equal(oa[:, :-1], ob[:, :-1]), day     # the BESS entry carries a's history
        assert a.get_scenarios()[0] == b.get_scenarios()[0]
        np.testing.assert_array_equal(a.pv_ratio(), b.pv_ratio())
        for t in range(24):
            a.step_tensors(torch.zeros((E, 11), device="cuda:0"))
            b.step_tensors(torch.zeros((E, 11), device="cuda:0"))
    a.close()
    b.close()


def test_sb3_vecenv_contract():
    """With SB3 importable (here: its abstract VecEnv stood in, tests/sb3_stub.py) the class is an SB3
    VecEnv, and seed() / set_options() apply at the next reset() and not at the automatic reset after a
    day, as DummyVecEnv does (SB3 2.x).  The days are those of the duck-typed class driven alike."""
    from sb3_stub import VecEnv, load_vec_env_with_sb3
    cls = load_vec_env_with_sb3().SmartNanogridVecEnv
    E = 64
    v = cls(E, seed=3, **KW)
    ref = SmartNanogridVecEnv(E, seed=50, **KW)
    assert isinstance(v, VecEnv) and v.reset_infos == [{}] * E and v.metadata == {"render_modes": ()}
    assert v.seed(50) == [50 + i for i in range(E)]
    np.testing.assert_array_equal(v.reset(), ref.reset())
    rng = np.random.default_rng(5)
    for t in range(24):
        if t == 23:
            v.seed(99)          # pending: the automatic reset below must not use it
        a = rng.uniform(0, 1, (E, 11)).astype(np.float32)
        o, r, d, info = v.step(a)
        o_ref, r_ref, d_ref, info_ref = ref.step(a)
        np.testing.assert_array_equal(o, o_ref)
        np.testing.assert_array_equal(r, r_ref)
        np.testing.assert_array_equal(d, d_ref)
    assert d.all() and all("terminal_observation" in i for i in info)
    np.testing.assert_array_equal(info[7]["terminal_observation"], info_ref[7]["terminal_observation"])
    # the pending seed 99 applies at this reset: the day of a fresh population seeded 99
    fresh = SmartNanogridVecEnv(E, seed=99, **KW)
    np.testing.assert_array_equal(v.reset()[:, :-1], fresh.reset()[:, :-1])   # BESS carries v's history
    assert v.get_scenarios()[0] == fresh.get_scenarios()[0]
    # options: the next reset() replays the day (generate_new_initial_values=False), then they are cleared
    v.set_options({"generate_new_initial_values": False})
    fresh.set_options({"generate_new_initial_values": False})
    day = v.get_scenarios()[0]
    v.reset()
    fresh.reset()
    np.testing.assert_array_equal(v.pv_ratio(), fresh.pv_ratio())
    assert [d["Arrivals"] for d in v.get_scenarios()[0]] == [d["Arrivals"] for d in day]
    assert v._options == [{}] * E and v.reset_infos == [{}] * E
    v.reset()
    assert v.get_scenarios()[0] != day
    for x in (v, ref, fresh):
        x.close()


def test_attributes_and_methods_per_index():
    E = 8
    v = SmartNanogridVecEnv(E, seed=4, **KW)
    v.reset()
    ratio = v.pv_ratio()
    assert v.get_attr("random_pv_shift_ratio", [1, 5]) == [ratio[1], ratio[5]]
    assert v.get_attr("number_of_chargers") == [10] * E
    assert v.get_attr("timestep", 3) == [0]
    with pytest.raises(AttributeError):
        v.get_attr("no_such_attribute")
    v.set_attr("battery_state_of_charge", 0.25, [1, 3])
    soc = v.battery_state_of_charge()
    assert soc[1] == soc[3] == 0.25 and soc[0] == soc[2] == 0.5
    with pytest.raises(ValueError):
        v.set_attr("algorithm_used", "PPO", [0])
    v.set_attr("algorithm_used", "PPO")
    assert v.get_attr("algorithm_used", [2]) == ["PPO"]
    res = v.env_method("get_scenario", indices=[2, 6])
    assert len(res) == 2 and res[0][1] == ratio[2] and res[1][1] == ratio[6]
    assert v.env_method("battery_state_of_charge", indices=[3]) == [0.25]
    with pytest.raises(ValueError):
        v.env_method("reset_tensors", indices=[0])
    assert len(v.env_method("pv_ratio")) == E
    with pytest.raises(IndexError):
        v.get_attr("random_pv_shift_ratio", [E])
    v.close()


def test_getters_report_errors_and_sync_the_callers_stream():
    E = 4096
    v = SmartNanogridVecEnv(E, seed=2, rng="device", **KW)
    s = torch.cuda.Stream()
    rc = lib().sng_get_battery_soc(v._h, None, ctypes.c_void_p(s.cuda_stream))
    assert rc == -1 and b"null host array" in lib().sng_last_error(v._h)
    rc = lib().sng_get_pv_ratio(v._h, None, None)
    assert rc == -1 and b"sng_get_pv_ratio" in lib().sng_last_error(v._h)
    # work queued on a side stream is seen by a getter ordered on that stream
    with torch.cuda.stream(s):
        _native.check(lib().sng_reset(v._h, _native.RNG_DEVICE, ctypes.c_void_p(v.obs_d.data_ptr()),
                                      ctypes.c_void_p(s.cuda_stream)), v._h)
        out = np.zeros(E)
        _native.check(lib().sng_get_pv_ratio(v._h, out.ctypes.data_as(_native.c_double_p),
                                             ctypes.c_void_p(s.cuda_stream)), v._h)
    assert set(np.unique(np.round(out * 100))).issubset(set(range(181))) and out.std() > 0
    v.close()


@pytest.mark.parametrize("N", [10, 33, 50, 128])
def test_device_days_draw_ratio_and_count_days_at_every_width(N):
    """wide stations took a generator path that left the PV ratio at 1.0 and the day counter
    advanced twice.  Every width must draw U{0..180}/100 ratios and advance the counter once a day."""
    E = 8192 if N <= 50 else 2048
    kw = dict(KW, number_of_chargers=N)
    v = SmartNanogridVecEnv(E, seed=9, rng="device", **kw)
    ratios = []
    for day in range(3):
        assert v.day_counter() == day
        v.reset_tensors()
        r = v.pv_ratio()
        ratios.append(r)
        assert set(np.unique(np.round(r * 100))).issubset(set(range(181)))
        assert abs(r.mean() - 0.9) < 0.05 and r.std() > 0.4
        for t in range(24):
            v.step_tensors(torch.zeros((E, N + 1), device="cuda:0"))
    assert v.day_counter() == 3
    assert not np.array_equal(ratios[0], ratios[1])
    v.close()


@pytest.mark.parametrize("N", [10, 50])
def test_device_reset_zeroes_the_injected_t0_penalty(N):
    """A day injected with a penalised vehicle in the python index -1 slot has a t = 0 penalty; the next
    device-RNG reset must start from 0 again (fused and separate t = 0 paths).  The twin runs the same
    injected day without that slot, so both advance the day counter alike."""
    E = 256
    kw = dict(KW, number_of_chargers=N, vehicle_uncharged_penalty_mode="dense")
    a = SmartNanogridVecEnv(E, seed=6, rng="device", **kw)
    b = SmartNanogridVecEnv(E, seed=6, rng="device", **kw)
    S = 25
    soc, occ, cap, req = (np.zeros((E, N, S)) for _ in range(4))
    occ[:, :, :5] = 1
    cap[:, :, :5] = 40
    soc[:, :, 0] = 0.5
    arr = np.zeros((E, N, 1), np.int32)
    dep = np.full((E, N, 1), 5, np.int32)
    soc_a, req_a = soc.copy(), req.copy()
    soc_a[:, :, 24] = 0.2
    req_a[:, :, 24] = 1.0                                     # python index -1: SOC 0.2, requested 1.0
    a.reset_from_arrays(soc_a, occ, cap, req_a, arr, dep, np.ones(E))
    b.reset_from_arrays(soc, occ, cap, req, arr, dep, np.ones(E))
    zero = torch.zeros((E, N + 1), device="cuda:0")
    _, r0, _ = a.step_tensors(zero)
    assert float(r0.max()) <= -64.0 * N + 1e-6                # the injected t = 0 penalty is there
    _, r0b, _ = b.step_tensors(zero)
    assert float(r0b.min()) > -64.0
    for t in range(1, 24):
        a.step_tensors(zero)
        b.step_tensors(zero)
    oa, ob = a.reset_tensors().clone(), b.reset_tensors().clone()
    assert torch.equal(oa, ob)
    _, ra, _ = a.step_tensors(zero)
    ra = ra.clone()
    _, rb, _ = b.step_tensors(zero)
    assert torch.equal(ra, rb)
    a.close()
    b.close()


def test_steps_only_graph_refuses_other_encodings():
    E, N = 512, 10
    kw = dict(KW, vehicle_uncharged_penalty_mode="dense")
    acts = torch.rand((24, E, N + 1), device="cuda:0")
    v = SmartNanogridVecEnv(E, seed=8, rng="reference", **kw)
    v.reset_tensors()
    iv, r = v.get_scenarios()
    for d in iv:   # a penalised requested SoC below 1: the injected day carries a requested-SoC stream
        d["Requested_SOC"] = [[0.9 if x else 0.0 for x in row] for row in d["Charger_occupancy"]]
    v.reset_from_initial_values(iv, r, restore_requested_soc=True)
    g = EpisodeGraph(v, acts, with_reset=False)
    v.reset_tensors()                   # reference RNG without requested SoC: no stream
    with pytest.raises(NativeError, match="another encoding"):
        g.launch()
    v.reset_from_initial_values(iv, r, restore_requested_soc=True)
    g.launch()                          # the same encoding again: allowed
    with pytest.raises(NativeError, match="t = 0"):
        g.launch()
    g.close()
    v.close()


def test_graphs_refuse_a_changed_seed():
    """a captured graph's kernels carry the seed and env offset by value; after seed() (or a
    restored state) has changed them, launching it would replay the old streams' days, so it refuses."""
    E, N = 512, 10
    acts = torch.rand((24, E, N + 1), device="cuda:0")
    v = SmartNanogridVecEnv(E, seed=4, rng="device", **KW)
    g = EpisodeGraph(v, acts, with_reset=True)
    g.launch()
    v.reset_tensors()
    s = EpisodeGraph(v, acts, with_reset=False)
    v.seed(5)
    v.reset_tensors()               # the seed applies here
    for gr in (g, s):
        with pytest.raises(NativeError, match="recapture"):
            gr.launch()
    g2 = EpisodeGraph(v, acts, with_reset=True)   # recaptured: the new seed's days
    g2.launch()
    for x in (g, s, g2, v):
        x.close()


def test_failed_injection_invalidates_the_day():
    """days are uploaded chunk by chunk as they are encoded; when a later env's day is
    refused, the earlier chunks have already overwritten the loaded day, so step / replay refuse until
    the next reset instead of stepping a half-replaced day."""
    E = 4096
    v = SmartNanogridVecEnv(E, seed=12, rng="reference", **KW)
    v.reset_tensors()
    iv, r = v.get_scenarios()
    bad = iv[-1]
    c = next(c for c in range(10) if any(bad["Charger_occupancy"][c]))
    t = bad["Charger_occupancy"][c].index(1.0)
    bad["Vehicle_capacities"][c][t] = 0.0          # an occupied slot with no battery: refused
    with pytest.raises(NativeError, match="reset again"):
        v.reset_from_initial_values(iv, r)
    with pytest.raises(NativeError, match="before reset"):
        v.step_tensors(torch.zeros((E, 11), device="cuda:0"))
    with pytest.raises(NativeError):
        v.replay_tensors()
    v.reset_tensors()
    v.step_tensors(torch.zeros((E, 11), device="cuda:0"))
    v.close()


def test_pending_seed_applies_to_graph_and_eager_days():
    """seed() left for the next reset applies at an EpisodeGraph of whole days (and run_eager_days /
    time_step_kernels), which begin with resets: the graph's day is a fresh population's first day of that
    seed.  A steps-only graph steps the loaded day, so it refuses while a seed waits."""
    E, N = 512, 10
    acts = torch.rand((24, E, N + 1), device="cuda:0")
    v = SmartNanogridVecEnv(E, seed=4, rng="device", **KW)
    v.reset_tensors()
    for t in range(24):
        v.step_tensors(acts[t])
    v.seed(5)
    with pytest.raises(ValueError, match="steps-only"):
        EpisodeGraph(v, acts, with_reset=False)
    g = EpisodeGraph(v, acts, with_reset=True)      # the seed applies here
    bess0 = v.battery_state_of_charge()
    g.launch()
    fresh = SmartNanogridVecEnv(E, seed=5, rng="device", **KW)
    fresh.set_battery_state_of_charge(bess0)
    fresh.reset_tensors()
    for t in range(24):
        fresh.step_tensors(acts[t])
    torch.testing.assert_close(v.return_d, fresh.return_d, rtol=0, atol=0)
    # and an eager day started by time_step_kernels after another seed()
    v.seed(6)
    v.time_step_kernels(acts, days=1)
    f6 = SmartNanogridVecEnv(E, seed=6, rng="device", **KW)
    f6.set_battery_state_of_charge(fresh.battery_state_of_charge())
    f6.reset_tensors()
    for t in range(24):
        f6.step_tensors(acts[t])
    torch.testing.assert_close(v.return_d, f6.return_d, rtol=0, atol=0)
    for x in (g, v, fresh, f6):
        x.close()


@pytest.mark.parametrize("rng", ["reference", "device"])
def test_load_state_discards_a_pending_seed(rng):
    """seed(s); load_state(blob); reset() continues the checkpoint's streams (its seed, RNG state
    and day counter) instead of re-seeding them at the reset."""
    E = 256
    a = SmartNanogridVecEnv(E, seed=21, rng=rng, **KW)
    a.reset_tensors()
    for t in range(24):
        a.step_tensors(torch.rand((E, 11), device="cuda:0"))
    blob = a.save_state()
    b = SmartNanogridVecEnv(E, seed=3, rng=rng, **KW)
    b.load_state(blob)
    a.seed(99)
    a.load_state(blob)
    oa, ob = a.reset_tensors().clone(), b.reset_tensors().clone()
    assert torch.equal(oa, ob)
    assert a.get_scenarios()[0] == b.get_scenarios()[0]
    a.close()
    b.close()


def test_flag_summary_reports_errors_and_v2x_breakpoints():
    """The numpy step() path watches the one-word flag summary (SngInfo.flag_summary) instead of a per-env
    flag store: a V2X station whose demand goes negative marks exactly the envs that hit the reference's
    breakpoint() (central_management_system.py:160-165) in infos, step after step, and a negative action on
    a non-V2X station raises the reference's ValueError (:158-159); the device path raises it at
    check_errors()."""
    E = 64
    v2x = dict(KW, vehicle_to_everything=True)
    v = SmartNanogridVecEnv(E, seed=2, rng="device", info=True, **v2x)   # per-env flags in the diagnostics too
    q = SmartNanogridVecEnv(E, seed=2, rng="device", **v2x)              # the default: summary word only
    v.reset()
    q.reset()
    rng = np.random.default_rng(1)
    seen = 0
    for t in range(24):
        a = np.zeros((E, 11), np.float32)
        a[:, :10] = -rng.random((E, 10))                  # everything discharges
        _, rv, _, iv = v.step(a)
        _, rq, _, iq = q.step(a)
        np.testing.assert_array_equal(rv, rq)
        flagged = v.last_info()["flags"] & _native.FLAG_V2X_BREAKPOINT
        got = np.array(["v2x_breakpoint" in d for d in iq])
        np.testing.assert_array_equal(got, flagged != 0)
        np.testing.assert_array_equal(got, np.array(["v2x_breakpoint" in d for d in iv]))
        seen += int(got.sum())
    assert seen > 0
    v.close()
    q.close()
    n = SmartNanogridVecEnv(E, seed=2, rng="device", **KW)
    n.reset()
    bad = np.zeros((E, 11), np.float32)
    with pytest.raises(ValueError, match="power_demand"):
        for t in range(24):
            bad[:, :10] = -1.0
            n.step(bad)
    n.reset_tensors()
    n.step_tensors(torch.from_numpy(bad).to(n.device))
    with pytest.raises(ValueError, match="power_demand"):
        n.check_errors()
    n.step_tensors(torch.zeros((E, 11), device=n.device))
    n.check_errors()   # cleared by the raise above: a clean step raises nothing
    n.close()


def test_injected_day_checks_the_python_stream_seed_in_device_mode():
    """a device-RNG env accepts a seed past numpy's range, but a day injected without pv_ratio draws
    each env's ratio from random.seed(seed + env_offset + i): refused in Python with a message naming the
    injected day, while an injected day with its ratios given works."""
    E = 4
    v = SmartNanogridVecEnv(E, seed=2 ** 32 - 2, rng="device", **KW)
    v.reset_tensors()
    iv, r = v.get_scenarios()
    with pytest.raises(ValueError, match="pv_ratio"):
        v.reset_from_initial_values(iv)
    obs = v.reset_from_initial_values(iv, r)
    assert np.isfinite(obs).all()
    # the library's own check (the blob's seed is unknown to Python after load_state) names the same cause
    blob = v.save_state()
    v.load_state(blob)
    with pytest.raises(NativeError, match="injected or replayed"):
        v.reset_from_initial_values(iv)
    v.close()


def test_load_state_rebuilds_the_flag_summary():
    """load_state replaces the sticky per-env flags, so the summary word follows them: a stale
    summary does not survive the restore, and V2X flags the blob holds unreported (raised on the device path)
    are reported at the next numpy step, for exactly the envs that raised them."""
    E = 64
    v2x = dict(KW, vehicle_to_everything=True)
    a = SmartNanogridVecEnv(E, seed=2, rng="device", **v2x)
    a.reset_tensors()
    act = torch.zeros((E, 11), device="cuda:0")
    act[: E // 2, :10] = -1.0   # the first half discharges: V2X demand < 0, flagged on the device
    a.step_tensors(act)
    pending = a.save_state()
    want = np.zeros(E, np.uint32)
    assert lib().sng_read_errors(a._h, want.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 0, None) == 0
    want = (want & _native.FLAG_V2X_BREAKPOINT) != 0
    assert want.any() and not want[E // 2:].any()
    b = SmartNanogridVecEnv(E, seed=9, rng="device", **v2x)
    b.reset_tensors()
    clean = b.save_state()
    b.flag_summary_d[7] = _native.FLAG_V2X_BREAKPOINT   # a stale summary from before the restore
    b.load_state(clean)
    assert not b.flag_summary_d.cpu().any()
    _, _, _, infos = b.step(np.zeros((E, 11), np.float32))
    assert not any("v2x_breakpoint" in d for d in infos)
    b.load_state(pending)
    assert int(np.bitwise_or.reduce(b.flag_summary_d.cpu().numpy())) & _native.FLAG_V2X_BREAKPOINT
    _, _, _, infos = b.step(np.zeros((E, 11), np.float32))   # no new flag: idle chargers
    got = np.array(["v2x_breakpoint" in d for d in infos])
    np.testing.assert_array_equal(got, want)
    _, _, _, infos = b.step(np.zeros((E, 11), np.float32))   # reported once: read and cleared
    assert not any("v2x_breakpoint" in d for d in infos)
    a.close()
    b.close()
