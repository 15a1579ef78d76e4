"""GPU: checkpoint / resume through the C ABI (sng_get_state / sng_set_state).

A day is stopped at t = 11, its state saved, and restored into a fresh handle created with another
seed; the restored handle finishes the day and runs the next one bit for bit like the uninterrupted
run (observations, rewards, dones, day returns, BESS and EV state of charge) -- for reference-RNG days
(the MT19937 streams travel in the blob, so the next day's draws match) and device-RNG days (the day
counter travels).  The state being carried is the reference's: EV SoC arrays (charger.py:16-19), the
BESS SoC and the day's initial SoC (central_management_system.py:93-94), the timestep
(smart_nanogrid_environment.py:312) and the loaded day.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smart_nanogrid_gym import SmartNanogridVecEnv  # noqa: E402
from smart_nanogrid_gym._native import NativeError  # noqa: E402


def run(v, acts, t0, days):
    out = []
    for d in range(days):
        if not (d == 0 and t0 > 0):
            v.reset_tensors()
        for t in range(t0 if d == 0 else 0, 24):
            o, r, dn = v.step_tensors(acts[d, t])
            out.append((o.clone(), r.clone(), dn.clone()))
        out.append((v.return_d.clone(),))
    return out


@pytest.mark.parametrize("rng,mode,req", [("reference", "sparse", False), ("reference", "dense", True),
                                          ("device", "sparse", False), ("device", "dense", True)])
def test_resume_mid_day_bit_exact(rng, mode, req):
    E, N = 1024, 10
    kw = dict(number_of_chargers=N, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode=mode, enable_requested_state_of_charge=req)
    g = torch.Generator(device="cuda:0").manual_seed(7)
    acts = torch.rand((2, 24, E, N + 1), generator=g, device="cuda:0")
    acts[..., -1] = acts[..., -1] * 2 - 1
    a = SmartNanogridVecEnv(E, seed=11, rng=rng, **kw)
    a.reset_tensors()
    for t in range(11):
        a.step_tensors(acts[0, t])
    blob = a.save_state()
    want = run(a, acts, 11, 2)
    want_state = (a.battery_state_of_charge(), a.vehicle_state_of_charge())
    b = SmartNanogridVecEnv(E, seed=999, rng=rng, **kw)   # another seed: the blob carries the streams
    b.load_state(blob)
    assert b.timestep == 11
    got = run(b, acts, 11, 2)
    assert len(got) == len(want)
    for x, y in zip(got, want):
        for p, q in zip(x, y):
            assert torch.equal(p, q)
    np.testing.assert_array_equal(b.battery_state_of_charge(), want_state[0])
    np.testing.assert_array_equal(b.vehicle_state_of_charge(), want_state[1])
    # the replayable day travels too
    assert torch.equal(a.replay_tensors(), b.replay_tensors())
    a.close()
    b.close()


def test_state_refuses_other_configuration():
    E = 256
    kw = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    a = SmartNanogridVecEnv(E, seed=1, **kw)
    a.reset_tensors()
    blob = a.save_state()
    for other in [dict(kw, vehicle_uncharged_penalty_mode="dense"), dict(kw, number_of_chargers=9)]:
        b = SmartNanogridVecEnv(E, seed=1, **other)
        with pytest.raises(NativeError, match="configuration"):
            b.load_state(blob)
        b.close()
    c = SmartNanogridVecEnv(E + 1, seed=1, **kw)
    with pytest.raises(NativeError):
        c.load_state(blob)
    with pytest.raises(NativeError):
        a.load_state(blob[:100])
    c.close()
    a.close()


def test_state_refuses_inconsistent_headers():
    """the header's section flags and size are checked against each other before any section
    is read (a corrupt blob must not drive reads past its end); the configuration fingerprint hashes the
    fields, so -0.0 and 0.0 are one configuration."""
    import struct
    E = 256
    kw = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    a = SmartNanogridVecEnv(E, seed=1, rng="reference", grid_cost_weight=0.0, **kw)
    a.reset_tensors()
    blob = a.save_state()
    total = struct.unpack_from("<Q", blob, 136)[0]
    assert total == len(blob)
    # StateHeader offsets: packed 72, has_word 112, has_req 116, has_prof 120, has_streams 128, total_bytes 136
    for off, fmt, val in [(112, "<i", 0), (128, "<i", 0), (120, "<i", 1), (72, "<i", 1), (116, "<i", 7),
                          (136, "<Q", total - 4 * 2 * 625 * E), (136, "<Q", 0)]:
        bad = bytearray(blob)
        struct.pack_into(fmt, bad, off, val)
        with pytest.raises(NativeError, match="corrupt state header"):
            a.load_state(bytes(bad))
    b = SmartNanogridVecEnv(E, seed=2, rng="reference", grid_cost_weight=-0.0, **kw)
    b.load_state(blob)
    assert torch.equal(a.replay_tensors(), b.replay_tensors())
    a.close()
    b.close()


def test_exported_streams_are_numpy_and_python_states():
    """The blob's stream section is numpy's RandomState state and Python's random state of every env (raw
    MT19937 words and position; the device keeps its blocks tempered, sng_layout.h RefStreams): after one
    reference-RNG reset, Python's stream is random.Random(seed + i) after the day's randint(0, 180)
    (smart_nanogrid_environment.py:349) and numpy's is RandomState(seed + i) some words further on."""
    import random
    E, seed = 32, 11
    kw = dict(number_of_chargers=4, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    a = SmartNanogridVecEnv(E, seed=seed, rng="reference", **kw)
    a.reset_tensors()
    blob = a.save_state()
    a.close()
    w = np.frombuffer(blob, dtype=np.uint32, count=E * 2 * 625, offset=len(blob) - E * 2 * 625 * 4).reshape(E, 2, 625)
    for i in range(E):
        r = random.Random(seed + i)
        r.randint(0, 180)
        st = r.getstate()[1]
        assert list(w[i, 1, :624]) == list(st[:624]) and int(w[i, 1, 624]) == st[624], i
        rs = np.random.RandomState(seed + i)
        for k in range(4000):   # the day drew k words: one 32-bit word per uint32 randint of full range
            _, key, pos = rs.get_state()[:3]
            if pos == int(w[i, 0, 624]) and np.array_equal(key, w[i, 0, :624]):
                break
            rs.randint(0, 2**32, dtype=np.uint32)
        else:
            raise AssertionError(f"env {i}: the exported numpy state is not RandomState({seed + i}) after any draw count")
        assert k > 0
