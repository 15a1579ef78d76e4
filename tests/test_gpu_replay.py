"""GPU: reset(generate_new_initial_values=False), the replay of the last generated day.

The reference replays through ChargingStation.load_initial_values (charging_station.py:119-136): the
day the last generation wrote to initial_values.json (:185-186) comes back with its vehicles, but
Requested_SOC stays at the 0 clear_initialisation_variables wrote (:138-150) -- so no vehicle is ever
penalised on a replayed day -- and reset() draws a new PV ratio (smart_nanogrid_environment.py:349).
solvers/evaluator.py:88-101 relies on it: the first model of an episode generates the day, the others
replay it.

* The reference's evaluator loop (evaluate_model_for_single_episode, evaluator.py:13-24, unchanged) on
  SmartNanogridEnv against fixtures made by running that loop on the reference itself
  (tests/golden/eval_*.npz, make_golden.py run_evaluator_case): observations bit-exact, rewards to
  1e-12 relative (the reference squares with libm pow, 1 ulp off x*x on ~0.1 % of inputs).
* Reference-RNG batches against the oracle's replay (x*x mode): bit-exact, several replays in a row.
* Device-RNG replays: the same vehicles, Requested_SOC 0, a new ratio, steps equal to the day injected
  with those arrays; replays do not move the device day counter.
* Misuse: replay with no generated day, or after an injected day; steps-only graphs across encodings.
"""
import ctypes

import numpy as np
import pytest

import oracle as O
from golden_util import eval_case, eval_cases

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from smart_nanogrid_gym import (EpisodeGraph, SmartNanogridEnv, SmartNanogridVecEnv,  # noqa: E402
                                evaluate_model_for_single_episode)
from smart_nanogrid_gym._native import NativeError  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _square_mode():
    O.lib().orc_set_square_mode.argtypes = [ctypes.c_int]
    O.lib().orc_set_square_mode(1)
    yield
    O.lib().orc_set_square_mode(0)


class RecordedModel:
    """A stand-in for a trained model: predict() returns the recorded actions of the current day and
    keeps the observations it was shown."""

    def __init__(self):
        self.actions, self.t, self.seen = None, 0, []

    def begin(self, day_actions):
        self.actions, self.t, self.seen = day_actions, 0, []

    def predict(self, obs):
        self.seen.append(np.array(obs, copy=True))
        a = self.actions[self.t]
        self.t += 1
        return a, None


@pytest.mark.parametrize("name", [m["name"] for m in eval_cases()])
def test_reference_evaluator_loop_unchanged(name):
    meta, d = eval_case(name)
    env = SmartNanogridEnv(seed=meta["seed"], **meta["kwargs"])
    models = [RecordedModel() for _ in range(meta["n_models"])]
    k = 0
    for ep in range(meta["n_episodes"]):            # solvers/evaluator.py:88-101
        reset_config = {"generate_new_initial_values": True}
        for model in models:
            reset_config["algorithm_used"] = "PPO"
            reset_config["environment_mode"] = "evaluation"
            model.begin(d["actions"][k])
            rewards = evaluate_model_for_single_episode(model, env, reset_config)
            assert len(rewards) == meta["T"]
            np.testing.assert_array_equal(model.seen[0], d["obs_reset"][k], err_msg=f"{name} day {k} reset")
            for t in range(1, meta["T"]):
                np.testing.assert_array_equal(model.seen[t], d["obs"][k][t - 1], err_msg=f"{name} day {k} t {t}")
            ref = d["reward"][k]
            assert np.all(np.abs(np.array(rewards) - ref) <= 1e-12 * np.maximum(1.0, np.abs(ref))), (name, k)
            reset_config["generate_new_initial_values"] = False
            k += 1
    env.close()


def test_reference_rng_batch_replays_vs_oracle():
    E, N, seed = 512, 10, 300
    kw = dict(number_of_chargers=N, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="dense", enable_requested_state_of_charge=True)
    venv = SmartNanogridVecEnv(E, seed=seed, rng="reference", info=True, **kw)
    cfg = O.OracleConfig(**kw)
    envs = [O.OracleEnv(cfg, seed + i) for i in range(E)]
    rng = np.random.default_rng(1)
    for kind in ["generate", "replay", "replay", "generate", "replay"]:
        if kind == "generate":
            obs = venv.reset_tensors().cpu().numpy()
            ref = np.stack([e.reset() for e in envs])
        else:
            obs = venv.replay_tensors().cpu().numpy()
            ref = np.stack([e.replay() for e in envs])
        np.testing.assert_array_equal(obs, ref, err_msg=kind)
        np.testing.assert_array_equal(venv.pv_ratio(), np.array([e.ratio for e in envs]))
        for t in range(24):
            a = rng.uniform(venv.action_space.low, venv.action_space.high, (E, venv.act_dim)).astype(np.float32)
            a[rng.random(a.shape) < 0.2] = 0
            o, r, _ = venv.step_tensors(torch.from_numpy(a).to(venv.device))
            outs = [e.step(a[i]) for i, e in enumerate(envs)]
            np.testing.assert_array_equal(o.cpu().numpy(), np.stack([x[0] for x in outs]), err_msg=f"{kind} t{t}")
            np.testing.assert_array_equal(r.cpu().numpy(), np.array([x[1] for x in outs]))
            pen = venv.last_info()["total_vehicle_penalty"]
            if kind == "replay":
                assert (pen == 0).all()
    venv.close()


def test_device_rng_replay():
    E, N = 2048, 10
    kw = dict(number_of_chargers=N, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="dense", enable_requested_state_of_charge=True)
    acts = torch.rand((3, 24, E, N + 1), device="cuda:0")
    acts[..., -1] = acts[..., -1] * 2 - 1
    a = SmartNanogridVecEnv(E, seed=5, rng="device", info=True, **kw)
    twin = SmartNanogridVecEnv(E, seed=5, rng="device", **kw)   # the same days without the replays
    o0 = a.reset_tensors().clone()
    twin.reset_tensors()
    iv0, r0 = a.get_scenarios()
    pen_gen = 0.0
    for t in range(24):
        a.step_tensors(acts[0, t])
        twin.step_tensors(acts[0, t])
        pen_gen += float(a.last_info()["total_vehicle_penalty"].sum())
    assert pen_gen > 0
    counter = a.day_counter()
    ratios = [r0]
    for rep in range(2):
        bess = a.battery_state_of_charge()
        o1 = a.replay_tensors().clone()
        iv1, r1 = a.get_scenarios()
        ratios.append(r1)
        for x, y in zip(iv0, iv1):   # the generated day's vehicles, Requested_SOC cleared
            for key in ("SOC", "Arrivals", "Departures", "Charger_occupancy", "Vehicle_capacities"):
                assert x[key] == y[key]
            assert np.all(np.array(y["Requested_SOC"]) == 0)
        assert set(np.unique(np.round(r1 * 100))).issubset(set(range(181)))
        np.testing.assert_array_equal(o1[:, 8:8 + 2 * N].cpu(), o0[:, 8:8 + 2 * N].cpu())   # SoC, departures
        # the replayed day steps like the same arrays injected into a fresh handle (BESS carried over)
        b = SmartNanogridVecEnv(E, seed=0, **kw)
        b.set_battery_state_of_charge(bess)
        ob = b.reset_from_initial_values(iv1, r1, restore_requested_soc=True)
        np.testing.assert_array_equal(ob, o1.cpu().numpy())
        for t in range(24):
            oa, ra, _ = a.step_tensors(acts[1 + rep, t])
            obb, rb, _ = b.step_tensors(acts[1 + rep, t])
            assert torch.equal(oa, obb) and torch.equal(ra, rb), (rep, t)
            assert float(np.abs(a.last_info()["total_vehicle_penalty"]).sum()) == 0.0
        b.close()
        assert a.day_counter() == counter   # a replay owns no day of the counter
    assert not np.array_equal(ratios[1], ratios[2]) and not np.array_equal(ratios[0], ratios[1])
    # the next generated day is the twin's second day (the BESS entry differs: a ran two more days)
    assert torch.equal(a.reset_tensors()[:, :-1], twin.reset_tensors()[:, :-1])
    (ia, ra), (it, rt) = a.get_scenarios(), twin.get_scenarios()
    assert ia == it and np.array_equal(ra, rt)
    a.close()
    twin.close()


def test_replay_misuse_and_graph_encodings():
    E, N = 1024, 10
    kw = dict(number_of_chargers=N, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    acts = torch.rand((24, E, N + 1), device="cuda:0")
    v = SmartNanogridVecEnv(E, seed=3, rng="device", **kw)
    with pytest.raises(NativeError, match="none was generated"):
        v.replay_tensors()
    v.reset_tensors()
    g_dev = EpisodeGraph(v, acts, with_reset=False)   # captured over a generated device day
    g_dev.launch()
    v.replay_tensors()
    with pytest.raises(NativeError, match="another encoding"):
        g_dev.launch()                                  # a replayed day: cleared Requested_SOC, no counter
    g_rep = EpisodeGraph(v, acts, with_reset=False)    # captured over the replayed day
    w = SmartNanogridVecEnv(E, seed=3, rng="device", **kw)
    w.reset_tensors()
    for t in range(24):
        w.step_tensors(acts[t])
    w.replay_tensors()
    g_rep.launch()
    for t in range(24):
        ow, rw, _ = w.step_tensors(acts[t])
    torch.cuda.synchronize()
    assert torch.equal(ow, v.obs_d) and torch.equal(rw, v.reward_d)
    with pytest.raises(NativeError, match="t = 0"):
        g_rep.launch()                                  # the day is over: a steps-only graph needs t = 0
    iv, r = v.get_scenarios()
    v.reset_from_initial_values(iv, r)
    with pytest.raises(NativeError, match="injected day"):
        v.replay_tensors()
    for x in (g_dev, g_rep, v, w):
        x.close()


def test_unstepped_device_day_replayed_is_counted_once():
    """a device day replayed before any of its steps was never counted (its first step counts
    it, a replay's steps do not); the next device reset must still draw a new day -- the day a twin that
    stepped the generated day draws next."""
    E, N = 512, 10
    kw = dict(number_of_chargers=N, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    acts = torch.rand((24, E, N + 1), device="cuda:0")
    v = SmartNanogridVecEnv(E, seed=21, rng="device", **kw)
    twin = SmartNanogridVecEnv(E, seed=21, rng="device", **kw)
    v.reset_tensors()
    twin.reset_tensors()
    day0 = v.get_scenarios()[0]
    assert v.day_counter() == 0
    v.replay_tensors()
    for t in range(24):
        v.step_tensors(acts[t])
        twin.step_tensors(acts[t])
    assert v.day_counter() == 1 == twin.day_counter()
    v.reset_tensors()
    twin.reset_tensors()
    day1 = v.get_scenarios()[0]
    assert day1 != day0 and day1 == twin.get_scenarios()[0]
    v.close()
    twin.close()
