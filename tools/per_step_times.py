"""Step-kernel device time by timestep (HIP events on every dispatch, eager device-RNG days).

    [SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_x.so] python tools/per_step_times.py

Prints the mean over 6 days of step 0, step 1 and steps 2-23 in microseconds, at 65,536 envs x
10 chargers: separates a cost that only the first step of a day pays (after the reset) from one
every step pays, when two builds are compared.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import torch  # noqa: E402

from smart_nanogrid_gym import SmartNanogridVecEnv  # noqa: E402


def main():
    E, N, days = 65536, 10, 6
    v = SmartNanogridVecEnv(E, seed=2024, rng="device", number_of_chargers=N, time_interval="1h",
                            charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    v._info.flags = None
    acts = torch.rand((24, E, N + 1), device="cuda:0")
    v.time_step_kernels(acts, days=2)   # warm-up
    us = v.time_step_kernels(acts, days=days).reshape(days, 24).mean(axis=0) * 1e3
    print(os.environ.get("SNG_LIBRARY", "libsng.so"),
          "t0 %.2f t1 %.2f t2-23 %.2f all %.3f us" % (us[0], us[1], us[2:].mean(), us.mean()))
    v.close()


if __name__ == "__main__":
    main()
