"""CPU: the lazily built per-env infos of SmartNanogridVecEnv.step_wait (vec_env.StepInfos).

DummyVecEnv returns a list of fresh dicts; StepInfos builds each env's dict on access.  These tests drive it
with the access patterns of SB3 2.x's own consumers (tests/sb3_stub.py restates them: VecMonitor,
the rollout's info buffer and timeout bootstrap, the off-policy transition store, the replay buffer's
timeouts, VecNormalize's in-place terminal observation) and compare with the plain list DummyVecEnv would
return.  The GPU side (terminal_observation bit-exact against the oracle) is tests/test_gpu_parity.py and
tests/test_gpu_vecenv_api.py."""
import copy
import pickle

import numpy as np
import pytest

import sb3_stub as S
from smart_nanogrid_gym.vec_env import StepInfos


def _plain(n, obs=None, done=None, v2x=()):
    out = [{} for _ in range(n)]
    if obs is not None:
        for i in range(n):
            if done[i]:
                out[i].update({"terminal_observation": obs[i], "TimeLimit.truncated": False})
    for i in v2x:
        out[i]["v2x_breakpoint"] = True
    return out


def _eq(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x.keys() == y.keys()
        for k in x:
            if isinstance(x[k], np.ndarray):
                assert np.array_equal(x[k], y[k])
            else:
                assert x[k] == y[k]


@pytest.mark.parametrize("case", ["running", "terminal", "mixed", "v2x"])
def test_step_infos_equal_dummy_vec_env_lists(case):
    n = 300
    rng = np.random.default_rng(1)
    obs = rng.random((n, 29)).astype(np.float32)
    done = {"running": None, "terminal": np.ones(n, bool), "mixed": rng.random(n) < 0.3, "v2x": None}[case]
    v2x = [3, 17, 299] if case in ("v2x", "mixed") else []
    args = (n, obs, done, v2x) if done is not None else (n, None, None, v2x)
    ref = _plain(*args)
    # every access pattern sees the same dicts
    _eq(list(StepInfos(*args)), ref)
    _eq([StepInfos(*args)[i] for i in range(n)], ref)
    _eq(StepInfos(*args)[:], ref)
    _eq(StepInfos(*args)[5:40:3], ref[5:40:3])
    _eq(StepInfos(*args)[-3:], ref[-3:])
    _eq(StepInfos(*args).copy(), ref)
    if done is None:   # (a list of dicts holding arrays has no == either)
        assert StepInfos(*args) == ref and StepInfos(*args) != ref[:-1]
    x = StepInfos(*args)
    assert len(x) == n and x[-1] is x[n - 1]
    with pytest.raises(IndexError):
        x[n]
    # a dict handed out by indexing is the one iteration yields later (writes persist)
    x = StepInfos(*args)
    x[7]["mine"] = 1
    _eq([list(x)[7]], [{**ref[7], "mine": 1}])
    assert x[7]["mine"] == 1 and list(x)[7] is x[7]
    # pickling and deep copies give the plain list
    for y in (pickle.loads(pickle.dumps(StepInfos(*args))), copy.deepcopy(StepInfos(*args))):
        assert type(y) is list
        _eq(y, ref)


def test_each_env_gets_its_own_dict():
    x = StepInfos(4)
    d = list(x)
    assert len({id(v) for v in d}) == 4 and all(v == {} for v in d)
    d[0]["a"] = 1
    assert x[1] == {} and x[0] == {"a": 1}


def test_sb3_consumers_see_dummy_vec_env_semantics():
    n, O = 64, 29
    rng = np.random.default_rng(2)
    returns, lengths = np.zeros(n), np.zeros(n, np.int64)
    returns2, lengths2 = np.zeros(n), np.zeros(n, np.int64)
    buf, buf2 = [], []
    for t in range(24):
        obs = rng.random((n, O)).astype(np.float32)
        rew = rng.random(n)
        done = np.full(n, t == 23)
        new_obs = rng.random((n, O)).astype(np.float32)
        lazy = StepInfos(n, obs, done) if done.any() else StepInfos(n)
        plain = _plain(n, obs, done) if done.any() else _plain(n)
        a = S.vec_monitor_step(rew, done, lazy, returns, lengths)
        b = S.vec_monitor_step(rew, done, plain, returns2, lengths2)
        _eq(a, b)
        S.update_info_buffer(a, done, buf)
        S.update_info_buffer(b, done, buf2)
        assert S.timeout_bootstrap_envs(done, lazy) == S.timeout_bootstrap_envs(done, plain) == []
        assert np.array_equal(S.store_transition_next_obs(new_obs, done, StepInfos(n, obs, done) if done.any()
                                                          else StepInfos(n)),
                              S.store_transition_next_obs(new_obs, done, plain))
        assert np.array_equal(S.replay_buffer_timeouts(lazy), S.replay_buffer_timeouts(plain))
    assert buf == buf2 and len(buf) == n
    # VecNormalize rewrites the done envs' terminal observation in place
    obs = rng.random((n, O)).astype(np.float32)
    done = np.ones(n, bool)
    lazy, plain = StepInfos(n, obs, done), _plain(n, obs, done)
    S.vec_normalize_terminal(done, lazy, 2.0)
    S.vec_normalize_terminal(done, plain, 2.0)
    _eq(list(lazy), plain)
    assert np.array_equal(lazy[5]["terminal_observation"], obs[5] * 2.0)
