"""Closed-loop throughput: a policy in the loop between the steps (not the headline bench).

bench.py replays days whose actions were generated beforehand.  Here every step's actions come
from the rule-based controller (solvers/RBC/rbc.py, smart_nanogrid_gym.RuleBasedController)
evaluated on the device observation tensor the previous step wrote -- the loop an RL rollout or
the reference's evaluator (solvers/evaluator.py:13-24) runs:

    obs = reset();  repeat T times: a = policy(obs); obs, r, done = step(a)

Policies (--policy): "rbc", the rule-based controller above (its torch form: round 5 removed the
controller's HIP kernel from libsng.so, SURVEY.md section 2 #20 puts it out of scope), or "mlp", the
network SB3's PPO("MlpPolicy", ...) builds by default (solvers/RL/ppo_train.py:89-92; net_arch 64-64,
tanh, deterministic predict = the action mean clipped to the Box), random-initialised in fp32 -- the
loop a PPO rollout or evaluation runs on this env, with torch's GEMMs (hipBLASLt) in it.

Two modes, one JSON line each:
  eager -- Python drives reset_tensors / policy / step_tensors (torch ops + C-ABI launches)
  graph -- the same day captured once with torch.cuda.graph and replayed (the C-ABI calls
           launch on torch's capturing stream, so the env kernels land in torch's graph)

    python tools/closed_loop_bench.py [--envs 65536] [--chargers 10] [--days 20] [--policy rbc|mlp]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import torch  # noqa: E402

from smart_nanogrid_gym import RuleBasedController, SmartNanogridVecEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--chargers", type=int, default=10)
    ap.add_argument("--days", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--policy", choices=("rbc", "mlp"), default="rbc")
    args = ap.parse_args()
    E, N = args.envs, args.chargers
    kw = dict(number_of_chargers=N, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse", pv_system_available_in_model=True,
              battery_system_available_in_model=True)
    venv = SmartNanogridVecEnv(E, seed=args.seed, rng="device", **kw)
    venv._info.flags = None
    if args.policy == "rbc":
        ctl = RuleBasedController(N)
        policy_desc = "RuleBasedController (solvers/RBC/rbc.py) on device obs"
    else:
        torch.manual_seed(args.seed)
        net = torch.nn.Sequential(torch.nn.Linear(venv.obs_dim, 64), torch.nn.Tanh(), torch.nn.Linear(64, 64),
                                  torch.nn.Tanh(), torch.nn.Linear(64, venv.act_dim)).to(venv.device)
        low = torch.tensor(venv.action_space.low, device=venv.device)
        high = torch.tensor(venv.action_space.high, device=venv.device)

        @torch.no_grad()
        def ctl(obs):
            return torch.maximum(torch.minimum(net(obs), high), low)
        policy_desc = "SB3 MlpPolicy-shaped actor (64-64 tanh, fp32, random init), action mean clipped to the Box"
    T = venv.timesteps
    total = torch.zeros(E, dtype=torch.float64, device=venv.device)

    def day():
        obs = venv.reset_tensors()
        for _ in range(T):
            obs, rew, _ = venv.step_tensors(ctl(obs))
        total.add_(venv.return_d)   # the day's returns, accumulated by the step kernel

    def timed(run, days):
        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(days):
            run()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    results = {}
    results["eager"] = timed(day, args.days)
    stream = torch.cuda.Stream(venv.device)
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):   # torch's warm-up for capture: allocator pools on this stream
        day()
    torch.cuda.current_stream().wait_stream(stream)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        day()
    results["graph"] = timed(graph.replay, args.days)
    r = total.cpu().numpy()
    assert (r == r).all() and (r <= 0).all()
    for mode, el in results.items():
        print(json.dumps({"metric": f"closed-loop env-steps/sec ({args.policy} policy in the loop)",
                          "mode": mode, "value": E * T * args.days / el, "unit": "env-steps/s",
                          "ms_per_day": el / args.days * 1e3, "envs": E, "chargers": N, "timesteps": T,
                          "days": args.days, "policy": policy_desc,
                          "reset": "device RNG", "data": "synthetic"}))
    venv.close()


if __name__ == "__main__":
    main()
