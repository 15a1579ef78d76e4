"""Can a device-RNG reset run under a day's steps?  Two independent handles on one GPU: A replays a steps-only
graph of one day (24 step kernels) on one stream, B runs device-RNG resets (generate_kernel) on another.
Times (device-synchronised wall, median of repeats): A alone, B alone, and both issued together.  If the
concurrent time is close to A alone, generating the next day's timeline while a day is stepped would hide the
reset; if it is close to A + B, the two kernels share the GPU and nothing is gained.

    python tools/overlap_probe.py [--envs 65536] [--days 20] [--repeats 5]
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

from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--days", type=int, default=20)
    ap.add_argument("--repeats", type=int, default=5)
    args = ap.parse_args()
    kw = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse")
    E, D = args.envs, args.days
    va = SmartNanogridVecEnv(E, seed=3, rng="device", **kw)
    vb = SmartNanogridVecEnv(E, seed=4, rng="device", **kw)
    T, A = va.timesteps, va.act_dim
    g = torch.Generator(device="cuda:0").manual_seed(1)
    acts = torch.rand((T, E, A), device="cuda:0", generator=g)
    acts[..., -1] = acts[..., -1] * 2 - 1
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(sa):
        va.reset_tensors()
        steps = EpisodeGraph(va, acts, with_reset=True, days=1)   # a day: reset + 24 steps
    torch.cuda.synchronize()

    def run_a():
        for _ in range(D):
            steps.launch(sa.cuda_stream)

    def run_b():
        with torch.cuda.stream(sb):
            for _ in range(D):
                vb.reset_tensors()

    def both():
        for _ in range(D):
            steps.launch(sa.cuda_stream)
            with torch.cuda.stream(sb):
                vb.reset_tensors()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        out = []
        for _ in range(args.repeats):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            out.append((time.perf_counter() - t0) * 1e3 / D)
        return round(float(np.median(out)), 4)

    res = {"envs": E, "days": D, "steps_day_ms": timed(run_a), "device_reset_ms": timed(run_b),
           "both_ms_per_day": timed(both)}
    res["hidden_fraction_of_reset"] = round((res["steps_day_ms"] + res["device_reset_ms"] - res["both_ms_per_day"])
                                            / res["device_reset_ms"], 3)
    print(json.dumps(res))
    steps.close()
    va.close()
    vb.close()


if __name__ == "__main__":
    main()
