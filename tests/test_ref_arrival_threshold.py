"""CPU: the integer arrival test of ref_day2_kernel (sng_kernels.hip kArrive53) against the reference's
double expression round(random.rand() - 0.1) == 1 (charging_station.py:214-215).

random.rand() is numpy's rk_double, K / 2^53 with K = (a >> 5) << 26 | (b >> 6) from two tempered words;
the kernel tests K >= 0x13333333333334 instead of computing the double.  Python's round() of a float
rounds half to even, so x = 0.5 does not arrive: arrival <=> fl(K / 2^53 - 0.1) > 0.5.
"""
import re
from pathlib import Path

import numpy as np

KERNELS = Path(__file__).resolve().parents[1] / "smart-nanogrid-gym_amd" / "csrc" / "sng_kernels.hip"


def _threshold():
    m = re.search(r"constexpr uint64_t kArrive53 = (0x[0-9a-fA-F]+)ull;", KERNELS.read_text())
    assert m, "kArrive53 not found in sng_kernels.hip"
    return int(m.group(1), 16)


def _arrives_double(k):
    return round(float(k) / 2.0**53 - 0.1) == 1


def test_threshold_is_the_first_arriving_draw():
    k = _threshold()
    assert _arrives_double(k) and not _arrives_double(k - 1)
    for d in range(-3000, 3001):
        assert _arrives_double(k + d) == (d >= 0), d


def test_threshold_on_random_word_pairs():
    k0 = _threshold()
    rng = np.random.default_rng(5)
    wa = rng.integers(0, 2**32, 200_000, dtype=np.uint64)
    wb = rng.integers(0, 2**32, 200_000, dtype=np.uint64)
    k = ((wa >> np.uint64(5)) << np.uint64(26)) | (wb >> np.uint64(6))
    r = (wa >> np.uint64(5)).astype(np.float64) * 67108864.0 + (wb >> np.uint64(6)).astype(np.float64)
    r /= 9007199254740992.0
    ref = np.round(r - 0.1) == 1   # numpy rounds half to even, as Python's round()
    assert np.array_equal(ref, k >= np.uint64(k0))
    assert abs(ref.mean() - 0.4) < 0.005
