"""Day time of the bench workload launched three ways on one stream, to separate the kernels' own time
from what a hipGraph adds between nodes: graph replays of 4 days (bench.py), eager C-side launches
without per-dispatch events (sng_time_step_kernels, ms = NULL), and eager launches with HIP start/stop
events on every dispatch.  HIP events around each mode on the same stream.

    python tools/launch_modes.py [days]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv  # noqa: E402


def main():
    days = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    E, N = 65536, 10
    venv = SmartNanogridVecEnv(E, seed=2024, rng="device", number_of_chargers=N, time_interval="1h",
                               charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    venv._info.flags = None
    g = torch.Generator(device="cuda:0").manual_seed(1)
    acts = torch.rand((24, E, N + 1), device="cuda:0", generator=g)
    acts[..., -1] = acts[..., -1] * 2 - 1
    acts = torch.where(torch.rand(acts.shape, device="cuda:0", generator=g) < 0.2, torch.zeros_like(acts), acts)
    venv.reset_tensors(rng="device")
    graph = EpisodeGraph(venv, acts, with_reset=True, days=4)

    def timed(fn):
        fn()   # warm-up
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / days, (time.perf_counter() - t0) * 1e6 / days

    res = {}
    res["graph x4"] = timed(lambda: [graph.launch() for _ in range(days // 4)])
    res["eager, no events"] = timed(lambda: venv.run_eager_days(acts, days))
    res["eager, events"] = timed(lambda: venv.time_step_kernels(acts, days))
    for k, (dev, wall) in res.items():
        print(f"{k:18s} device {dev:8.2f} us/day   wall {wall:8.2f} us/day")
    graph.close()
    venv.close()


if __name__ == "__main__":
    main()
