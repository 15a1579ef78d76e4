"""Throughput of the path stable-baselines3 drives: SmartNanogridVecEnv.step(np.ndarray) -> (obs, rewards,
dones, infos) with numpy actions in and numpy results out, automatic reset at the end of every day, on the
default reference RNG (solvers/RL/ppo_train.py:89-102 hands the env to PPO, whose collect_rollouts calls
env.step(clipped_actions) once per rollout step).

    python tools/sb3_path_bench.py [--envs 65536] [--days 20] [--rng reference|device] [--consume]

Prints one JSON line: env-steps/s over whole days (the 24 steps of each day, its automatic reset included),
and the split of one step into its phases, each the median over the timed steps:
  actions_in  np.asarray + copy into the pinned actions buffer (host)
  h2d         the pinned -> device copy of the actions (HIP events)
  step        the step kernel (HIP events)
  d2h         the device -> pinned copy of the step's outputs (HIP events)
  sync        host time from the last enqueue until the stream is done
  host_out    the flag check and the host copies of the results
  reset       the automatic reset of a done step, per day: reset_enqueue (the reset and its observation's
              D2H copy queued), terminal_infos (the 65,536 terminal_observation infos, built while the
              device resets), reset_wait (what is left of the device's work), reset_copy (the new day's
              observations to a fresh array); reset_device = the reset + copy on the device (HIP events)
Synthetic actions: uniform in the action Box, 20 % exact zeros, pre-generated host arrays (as a policy's
numpy output arrives).  Steps are driven exactly as SB3 does, one env.step() per rollout step.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--chargers", type=int, default=10)
    ap.add_argument("--days", type=int, default=20, help="timed days")
    ap.add_argument("--warmup-days", type=int, default=1)
    ap.add_argument("--rng", default="reference", choices=["reference", "device"])
    ap.add_argument("--pkg", default=None, help="A/B: the directory holding another smart_nanogrid_gym package")
    ap.add_argument("--consume", action="store_true",
                    help="after every step, read the infos as SB3 2.x's PPO rollout does (its info buffer update "
                         "over every env's info and the timeout-bootstrap check; tests/sb3_stub.py restates both) "
                         "and time that as `consumer_ms_per_step`")
    args = ap.parse_args()
    if args.pkg:
        sys.path.insert(0, os.path.abspath(args.pkg))
    from smart_nanogrid_gym import SmartNanogridVecEnv
    kw = dict(number_of_chargers=args.chargers, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse", pv_system_available_in_model=True,
              battery_system_available_in_model=True)
    E = args.envs
    venv = SmartNanogridVecEnv(E, seed=7, rng=args.rng, **kw)
    T, A = venv.timesteps, venv.act_dim
    rng = np.random.default_rng(0)
    lo, hi = venv.action_space.low, venv.action_space.high
    pool = []
    for _ in range(4):
        a = (lo + (hi - lo) * rng.random((E, A))).astype(np.float32)
        a[rng.random(a.shape) < 0.2] = 0.0
        pool.append(a)
    venv.reset()
    for i in range(args.warmup_days * T):
        venv.step(pool[i % len(pool)])
    if args.consume:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import sb3_stub as S
    consumer = []
    ep_buf = []
    venv.profile_phases(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = args.days * T
    for i in range(n):
        obs, rew, done, infos = venv.step(pool[i % len(pool)])
        if args.consume:
            tc = time.perf_counter()
            S.update_info_buffer(infos, done, ep_buf)
            S.timeout_bootstrap_envs(done, infos)
            consumer.append(time.perf_counter() - tc)
    elapsed = time.perf_counter() - t0
    ph = venv.profile_phases(False)
    assert obs.shape == (E, venv.obs_dim) and np.isfinite(rew).all() and len(infos) == E
    split = {k: round(float(np.median(v)) * 1e3, 4) for k, v in ph.items() if v}
    out = {"metric": "env-steps/s through SmartNanogridVecEnv.step(np.ndarray) (the SB3 path)",
           "value": E * n / elapsed, "unit": "env-steps/s", "envs": E, "chargers": args.chargers,
           "timesteps": T, "days": args.days, "rng": args.rng, "ms_per_step": elapsed / n * 1e3,
           "split_ms_median": split,
           "note": "reset* are per day (one automatic reset per 24 steps); every other phase per step",
           "reset_ms_per_day_mean": round(float(np.mean(ph["reset"])) * 1e3, 4) if ph.get("reset") else None,
           "consumer_ms_per_step": round(float(np.mean(consumer)) * 1e3, 4) if consumer else None,
           "value_without_consumer": (E * n / (elapsed - sum(consumer))) if consumer else None}
    print(json.dumps(out))
    venv.close()


if __name__ == "__main__":
    main()
