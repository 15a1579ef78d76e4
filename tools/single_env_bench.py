"""Per-call latency of the one-env drop-in path: SmartNanogridEnv.step(np.ndarray) and reset(), as
solvers/RL/ppo_train.py:89-92 (gym.make -> SB3's DummyVecEnv, one env.step per policy step) and
solvers/evaluator.py:13-24 (the 5-tuple loop) call them, unchanged.

    python tools/single_env_bench.py [--days 1000] [--chargers 10] [--rng reference|device]

Prints one JSON line: the median / p90 / mean per-call microseconds of step() and reset() over `days` whole
days (24 steps each at 1 h), and the env-steps/s of the loop (reset included).  Actions: uniform in the
action Box with 20 % exact zeros, pre-generated numpy arrays (as a policy's output arrives).  The reference's
own step() (~183 us per step on this container's Xeon, pure Python, JSON I/O
stubbed) is the figure this path replaces; `reference_step_us` quotes it.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import numpy as np  # noqa: E402

REFERENCE_STEP_US = 183.0   # SURVEY.md section 8a R4 (reference step(), N = 10, cProfile, I/O stubbed)
REFERENCE_RESET_US = (400.0, 800.0)


def stats(x):
    x = np.asarray(x) * 1e6
    return {"median": round(float(np.median(x)), 2), "p90": round(float(np.percentile(x, 90)), 2),
            "mean": round(float(x.mean()), 2), "min": round(float(x.min()), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=int, default=1000)
    ap.add_argument("--warmup-days", type=int, default=20)
    ap.add_argument("--chargers", type=int, default=10)
    ap.add_argument("--rng", default="reference", choices=["reference", "device"])
    ap.add_argument("--path", default=None, help="SmartNanogridEnv step path (A/B: 'host' or 'torch')")
    args = ap.parse_args()
    from smart_nanogrid_gym import SmartNanogridEnv
    kw = dict(number_of_chargers=args.chargers, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse", pv_system_available_in_model=True,
              battery_system_available_in_model=True)
    env = SmartNanogridEnv(seed=11, rng=args.rng, **kw)
    if args.path is not None:
        env.step_path = args.path
    T = env._venv.timesteps
    rng = np.random.default_rng(0)
    lo, hi = env.action_space.low, env.action_space.high
    pool = (lo + (hi - lo) * rng.random((4096, lo.size))).astype(np.float32)
    pool[rng.random(pool.shape) < 0.2] = 0.0
    k = 0
    for _ in range(args.warmup_days):
        env.reset()
        for _ in range(T):
            env.step(pool[k % len(pool)])
            k += 1
    step_s, reset_s = [], []
    ret = 0.0
    t_start = time.perf_counter()
    for _ in range(args.days):
        t0 = time.perf_counter()
        obs, _ = env.reset()
        reset_s.append(time.perf_counter() - t0)
        done = False
        while not done:
            a = pool[k % len(pool)]
            k += 1
            t0 = time.perf_counter()
            obs, r, done, trunc, info = env.step(a)
            step_s.append(time.perf_counter() - t0)
            ret += r
    elapsed = time.perf_counter() - t_start
    assert len(step_s) == args.days * T and np.isfinite(ret)
    out = {"metric": "per-call latency of SmartNanogridEnv.step / reset (the one-env drop-in path)",
           "chargers": args.chargers, "timesteps": T, "days": args.days, "rng": args.rng,
           "step_path": getattr(env, "step_path", None),
           "step_us": stats(step_s), "reset_us": stats(reset_s),
           "env_steps_per_s": args.days * T / elapsed,
           "reference_step_us": REFERENCE_STEP_US, "reference_reset_us": list(REFERENCE_RESET_US),
           "speedup_vs_reference_step_median": round(REFERENCE_STEP_US / (np.median(step_s) * 1e6), 2)}
    print(json.dumps(out))
    env.close()


if __name__ == "__main__":
    main()
