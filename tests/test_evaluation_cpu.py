"""CPU: the reference's callers restated in smart_nanogrid_gym.evaluation -- the rule-based
controller (solvers/RBC/rbc.py:4-29) batched in torch vs its row-by-row form, and the
evaluator / predictor episode loops (solvers/evaluator.py:13-24, predictor.py:14-25) on a
stand-in env with the 5-tuple API."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from smart_nanogrid_gym.evaluation import (RuleBasedController, evaluate_model_for_single_episode,  # noqa: E402
                                           predict_single_day)


def _obs(rng, B, N, bess=True):
    O = 8 + 2 * N + (1 if bess else 0)
    obs = rng.uniform(0, 1.8, (B, O)).astype(np.float32)
    dep = rng.integers(0, 11, (B, N)).astype(np.float32) / np.float32(24)
    dep[:, 0] = np.float32(4 / 24)          # 0.1666667 < 0.16667: leaving soon
    dep[:, 1 % N] = np.float32(0.16667)     # on the threshold: follows the PV forecast
    obs[:, 8 + N:8 + 2 * N] = dep
    return obs


@pytest.mark.parametrize("N,bess", [(1, True), (4, False), (10, True), (50, True)])
def test_rule_based_controller_batched_equals_rows(N, bess):
    rng = np.random.default_rng(N)
    obs = _obs(rng, 257, N, bess)
    ctl = RuleBasedController(N, True, bess)
    batched = ctl(torch.from_numpy(obs)).numpy()
    rows = np.stack([ctl.select_action(o) for o in obs])
    assert batched.dtype == np.float32 and batched.shape == (257, N + (1 if bess else 0))
    np.testing.assert_array_equal(batched, rows)
    np.testing.assert_array_equal(ctl.predict(obs)[0], rows)
    np.testing.assert_array_equal(ctl.predict(obs[3])[0], rows[3])


def test_rule_based_controller_rule():
    """rbc.py:12-27 case by case (departure at index 8 + N + c of this env's observation)."""
    N = 3
    ctl = RuleBasedController(N)
    s = np.zeros(8 + 2 * N + 1, np.float32)
    s[0], s[2] = 0.5, 1.25                                  # solar(t), solar(t+1)
    s[8 + N:8 + 2 * N] = [0.0, 3 / 24, 9 / 24]
    np.testing.assert_array_equal(ctl.select_action(s), np.float32([0.0, 1.0, 0.875, 0.0]))
    with pytest.raises(ValueError):
        RuleBasedController(N, pv_system_available_in_model=False)


class _CountdownEnv:
    """5-tuple gym env stand-in: T steps, reward = -(sum of the action) - t."""

    def __init__(self, T):
        self.T, self.t, self.resets = T, 0, []

    def reset(self, **kwargs):
        self.resets.append(kwargs)
        self.t = 0
        return np.zeros(3, np.float32), {}

    def step(self, a):
        r = -float(np.sum(a)) - self.t
        self.t += 1
        return np.full(3, self.t, np.float32), r, self.t == self.T, False, {}


class _EchoModel:
    def predict(self, obs):
        return obs[:2] + 1, None


def test_episode_loops():
    env = _CountdownEnv(5)
    kw = {"generate_new_initial_values": True, "algorithm_used": "PPO", "environment_mode": "evaluation"}
    r = evaluate_model_for_single_episode(_EchoModel(), env, kw)
    assert r == [-(2 * (t + 1)) - t for t in range(5)]
    assert env.resets == [kw]
    assert predict_single_day(_EchoModel(), env, {}) == r
