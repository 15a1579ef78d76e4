"""The reference's callers of the environment, over the batched GPU implementation.

The reference drives its env from three small loops (solvers/):
  * evaluator.py:13-24   evaluate_model_for_single_episode(model, env, kwargs)
  * predictor.py:14-25   predict_single_day(model, env, kwargs) (also predictor_class.py:38-48)
  * evaluator.py:80-106  every model plays the same `episodes` days (the first model's reset
                         generates the day, the others replay it with
                         generate_new_initial_values=False); per-model episode totals and means
and ships a rule-based controller, solvers/RBC/rbc.py:4-29.

`evaluate_model_for_single_episode` / `predict_single_day` are the same loops for the
single-env `SmartNanogridEnv` (5-tuple API), unchanged.  `evaluate_models` is the batched form
of evaluator.py:80-106: all models x episodes run as one env population on the GPU, one fused
step kernel per timestep for all of them, with each model's policy evaluated on its slice of the
device observation tensor.  `RuleBasedController` restates rbc.py's rule on this env's
observation layout, batched in torch (it runs on the device tensors, or on numpy rows).

Differences from the reference scripts (deliberate, documented):
  * Every (model, episode) slot starts the day with the same battery state of charge
    (`battery_initial_soc`, default the config's); the reference's evaluator shares ONE env per
    variant, so each model's episode inherits the battery its predecessor left.
  * Replayed days keep the generating day's PV shift ratio and requested SoC.  The reference redraws
    the ratio from the global `random` stream at every reset, replays included
    (smart_nanogrid_environment.py:349), and its replays leave Requested_SOC at 0
    (charging_station.py:119-136).  The unchanged single-env loop above reproduces that exactly:
    SmartNanogridEnv.reset(generate_new_initial_values=False) replays the env's last generated day.
"""

import numpy as np

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


# ----------------------------------------------------------------------------- single-env loops
def evaluate_model_for_single_episode(current_model, env, kwargs):
    """solvers/evaluator.py:13-24: one episode with `current_model.predict(obs)`; the per-step rewards."""
    rewards_list = []
    obs, _ = env.reset(**kwargs)
    done = False
    while not done:
        action, _states = current_model.predict(obs)
        obs, reward, terminated, truncated, info = env.step(action)
        done = terminated or truncated
        rewards_list.append(reward)
    return rewards_list


def predict_single_day(current_model, env, kwargs):
    """solvers/predictor.py:14-25 (predictor_class.py:38-48): the same loop as the evaluator."""
    return evaluate_model_for_single_episode(current_model, env, kwargs)


# ----------------------------------------------------------------------------- rule-based control
class RuleBasedController:
    """solvers/RBC/rbc.py:4-29 on this environment's observation layout.

    Per charger c, from the normalised remaining time to departure d_c (observation entry
    `k + N + c`, k = 8 with PV):
        d_c == 0              -> 0                     (no vehicle)
        0 < d_c < 0.16667     -> 1                     (leaves within 4 h: charge at full power)
        otherwise             -> (solar[t] + solar[t+1]) / 2   (observation entries 0 and 2)
    The BESS action (battery variants) is 0.  As in rbc.py nothing is clipped: the solar terms
    carry the PV shift ratio and can exceed 1.  The rule reads the PV forecast, so variants
    without PV are rejected.

    `controller(obs)` maps a [B, obs_dim] torch tensor (any device) to [B, act_dim] float32
    actions on the same device; `select_action(states)` takes one observation row (numpy), as
    rbc.py does; `predict(obs)` is the stable-baselines-style (actions, None) pair.
    """

    LEAVING_SOON = 0.16667   # rbc.py:16 (4 h of the /24 departure scale)

    def __init__(self, number_of_chargers, pv_system_available_in_model=True,
                 battery_system_available_in_model=True):
        if not pv_system_available_in_model:
            raise ValueError("the rule-based controller follows the PV forecast: needs a PV variant")
        self.NUMBER_OF_CHARGERS = int(number_of_chargers)
        self.bess = bool(battery_system_available_in_model)
        self.k_dep = 8 + self.NUMBER_OF_CHARGERS   # [solar, price, solar x3, price x3, SoC x N, departure x N, (bess)]
        self.act_dim = self.NUMBER_OF_CHARGERS + (1 if self.bess else 0)

    @classmethod
    def for_env(cls, env):
        s = env.settings if hasattr(env, "settings") else env._venv.settings
        return cls(s.number_of_chargers, s.pv_system_available_in_model, s.battery_system_available_in_model)

    def select_action(self, states):
        """rbc.py:6-29 for one observation row."""
        states = np.asarray(states)
        action = [0.0] * self.act_dim
        for car in range(self.NUMBER_OF_CHARGERS):
            d = states[self.k_dep + car]
            if d == 0:
                action[car] = 0
            elif 0 < d < self.LEAVING_SOON:
                action[car] = 1
            else:
                action[car] = (states[0] + states[2]) / 2
        return np.asarray(action, dtype=np.float32)

    def __call__(self, obs):
        N = self.NUMBER_OF_CHARGERS
        d = obs[:, self.k_dep:self.k_dep + N]
        follow = ((obs[:, 0:1] + obs[:, 2:3]) / 2).expand(-1, N)
        a = torch.where(d == 0, torch.zeros_like(d),
                        torch.where((d > 0) & (d < self.LEAVING_SOON), torch.ones_like(d), follow))
        if self.bess:
            a = torch.cat([a, torch.zeros_like(a[:, :1])], dim=1)
        return a.to(torch.float32)

    def predict(self, obs, state=None, episode_start=None, deterministic=True):
        obs = np.asarray(obs, dtype=np.float32)
        if obs.ndim == 1:
            return self.select_action(obs), None
        return self(torch.from_numpy(obs)).numpy(), None


# ----------------------------------------------------------------------------- batched evaluator
def _policy_actions(policy, obs_d):
    """Device actions from a policy: a torch callable on the device tensor, or an object with a
    stable-baselines-style predict(numpy obs batch) -> (actions, state)."""
    if hasattr(policy, "predict") and not isinstance(policy, RuleBasedController):
        a, _ = policy.predict(obs_d.cpu().numpy())
        return torch.as_tensor(np.asarray(a, np.float32), device=obs_d.device)
    return policy(obs_d)


def generate_days(episodes, *, seed=0, device=0, rng="reference", **env_kwargs):
    """`episodes` new days as the reference's initial_values dicts plus their PV ratios (env i of a
    population seeded `seed` -- with rng='reference' the day env i of SmartNanogridVecEnv(seed=seed)
    or the reference after np.random.seed(seed + i); random.seed(seed + i) would generate)."""
    from .vec_env import SmartNanogridVecEnv
    gen = SmartNanogridVecEnv(episodes, seed=seed, device=device, rng=rng, **env_kwargs)
    try:
        gen.reset_tensors()
        torch.cuda.current_stream(gen.device).synchronize()
        ivs, ratios = gen.get_scenarios(0, episodes)
    finally:
        gen.close()
    return ivs, ratios


def evaluate_models(models, episodes=100, *, seed=0, device=0, rng="reference", battery_initial_soc=None,
                    days=None, **env_kwargs):
    """solvers/evaluator.py:80-106, batched: every model plays the same `episodes` days.

    models -- {name: policy}; a policy is a torch callable [B, obs_dim] -> [B, act_dim] on the
              device tensors, or has predict(numpy obs batch) -> (actions, state)
    days   -- optional (initial_values list, pv ratios) from generate_days(); generated otherwise
    Returns (final_rewards {name: float64[episodes]} = per-episode total reward,
             mean_rewards {name: float}), as evaluator.py:85-106 builds them.
    """
    from .vec_env import SmartNanogridVecEnv
    names = list(models)
    if days is None:
        days = generate_days(episodes, seed=seed, device=device, rng=rng, **env_kwargs)
    initial_values, ratios = days
    episodes = len(initial_values)
    M = len(names)
    venv = SmartNanogridVecEnv(M * episodes, seed=seed, device=device, rng=rng, **env_kwargs)
    try:
        if battery_initial_soc is not None:
            venv.set_battery_state_of_charge(battery_initial_soc)
        venv.reset_from_initial_values(list(initial_values) * M, np.tile(ratios, M), restore_requested_soc=True)
        obs = venv.obs_d
        actions = torch.empty((M * episodes, venv.act_dim), dtype=torch.float32, device=venv.device)
        totals = torch.zeros(M * episodes, dtype=torch.float64, device=venv.device)
        for _ in range(venv.timesteps):
            for m, name in enumerate(names):
                sl = slice(m * episodes, (m + 1) * episodes)
                actions[sl] = _policy_actions(models[name], obs[sl])
            obs, rew, _ = venv.step_tensors(actions)
            totals += rew
        venv.check_errors()   # the reference's errors of any step of the day, as step() raises them
        totals = totals.cpu().numpy().reshape(M, episodes)
    finally:
        venv.close()
    final_rewards = {name: totals[m] for m, name in enumerate(names)}
    mean_rewards = {name: float(np.mean(totals[m])) for m, name in enumerate(names)}
    return final_rewards, mean_rewards
