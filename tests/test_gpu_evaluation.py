"""GPU: the reference's callers (smart_nanogrid_gym.evaluation) in closed loop on the device.

* evaluate_model_for_single_episode (solvers/evaluator.py:13-24) with the rule-based controller
  (solvers/RBC/rbc.py) on SmartNanogridEnv: per-step rewards bit-exact against the CPU oracle
  driven by the same controller on the oracle's own observations (x*x square mode).
* evaluate_models (the batched evaluator.py:80-106): every model plays the same days; each
  (model, episode) total equals a direct VecEnv run of that day with that policy (the day
  re-injected from its decoded initial values must step bit for bit like the generated one) and,
  for reference-RNG days, the oracle's episode total.
"""
import ctypes

import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smart_nanogrid_gym import (RuleBasedController, SmartNanogridEnv, SmartNanogridVecEnv,  # noqa: E402
                                evaluate_model_for_single_episode, evaluate_models, generate_days)

KW = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse",
          pv_system_available_in_model=True, battery_system_available_in_model=True)


@pytest.fixture(scope="module", autouse=True)
def _square_mode():
    O.lib().orc_set_square_mode.argtypes = [ctypes.c_int]
    O.lib().orc_set_square_mode(1)
    yield
    O.lib().orc_set_square_mode(0)


def _zeros(obs):
    return torch.zeros((obs.shape[0], 11), dtype=torch.float32, device=obs.device)


def _full(obs):
    a = torch.ones((obs.shape[0], 11), dtype=torch.float32, device=obs.device)
    a[:, -1] = -0.5   # discharge the battery a little every step
    return a


def _oracle_episode(policy_rows, seed, days=1):
    cfg = O.OracleConfig(**KW)
    env = O.OracleEnv(cfg, seed)
    out = []
    for _ in range(days):
        obs = env.reset()
        rewards = []
        for _t in range(24):
            obs, r = env.step(policy_rows(obs))[:2]
            rewards.append(r)
        out.append(rewards)
    return out


def test_rbc_single_episode_vs_oracle():
    ctl = RuleBasedController(10)
    env = SmartNanogridEnv(seed=77, **KW)
    got = [evaluate_model_for_single_episode(ctl, env, {"algorithm_used": "RBC"}) for _ in range(3)]
    env.close()
    ref = _oracle_episode(ctl.select_action, 77, days=3)
    assert [len(r) for r in got] == [24, 24, 24]
    np.testing.assert_array_equal(np.array(got), np.array(ref))


@pytest.mark.parametrize("rng", ["reference", "device"])
def test_evaluate_models_same_days(rng):
    episodes, seed = 16, 4242
    ctl = RuleBasedController(10)
    models = {"rbc": ctl, "zeros": _zeros, "full": _full}
    days = generate_days(episodes, seed=seed, rng=rng, **KW)
    final, mean = evaluate_models(models, days=days, seed=seed, rng=rng, **KW)
    assert set(final) == set(models) and all(v.shape == (episodes,) for v in final.values())
    for name, pol in models.items():
        assert mean[name] == pytest.approx(float(np.mean(final[name])), rel=0, abs=0)
        # the same days, generated (not injected) by a population with the same seed
        venv = SmartNanogridVecEnv(episodes, seed=seed, rng=rng, **KW)
        obs = venv.reset_tensors()
        tot = torch.zeros(episodes, dtype=torch.float64, device=venv.device)
        for _t in range(24):
            obs, rew, _ = venv.step_tensors(pol(obs))
            tot += rew
        venv.close()
        np.testing.assert_array_equal(final[name], tot.cpu().numpy())
    if rng == "reference":   # and against the oracle's episodes (env i = reference seeded seed + i)
        for i in (0, 5, episodes - 1):
            ref = _oracle_episode(ctl.select_action, seed + i)[0]
            assert final["rbc"][i] == sum(ref)   # both sum the day's rewards left to right in f64
    assert mean["full"] != mean["zeros"]
