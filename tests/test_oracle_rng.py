"""The oracle's MT19937 restatement, draw for draw against numpy's legacy RandomState and
Python's random module (the two global streams the reference's reset() consumes)."""
import random

import numpy as np
import pytest

import oracle as O


@pytest.mark.parametrize("seed", [0, 1, 13, 2**31 + 5, 4294967295])
def test_numpy_legacy_stream(seed):
    rs = np.random.RandomState(seed)
    o = O.OracleRng(seed)
    for i in range(3000):
        k = i % 4
        if k == 0:
            assert o.random() == rs.rand()
        elif k == 1:
            assert o.uniform(0.1, 0.9) == rs.uniform(0.1, 0.9)
        elif k == 2:
            assert o.np_randint(15, 120) == rs.randint(15, 120)
        else:
            lo = i % 23
            hi = lo + 1 + (i % 7)
            assert o.np_randint(lo, hi) == rs.randint(lo, hi)   # includes single-value ranges (no draw)


@pytest.mark.parametrize("seed", [0, 7, 123456789, 2**40 + 3])
def test_python_random_stream(seed):
    r = random.Random(seed)
    o = O.OracleRng(seed, python_style=True)
    for _ in range(2000):
        assert o.py_randint(0, 180) == r.randint(0, 180)


def test_pairwise_sum_matches_numpy():
    rng = np.random.default_rng(3)
    for n in list(range(0, 40)) + [127, 128, 129, 200, 257, 1000]:
        a = rng.random(n) * np.exp(rng.normal(0, 4, n))
        assert O.pairwise_sum(a) == a.sum()
