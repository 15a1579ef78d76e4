"""Time the reference-RNG reset (sng_reset(SNG_RNG_REFERENCE): host MT19937 days on the host threads,
encoded into pinned staging and uploaded chunk by chunk while the next chunk is built) and the other
resets, at 4,096 and 65,536 envs x 10 chargers.  This is the reset SB3 auto-reset runs every day with
the VecEnv default rng='reference' (vec_env.py step_wait).

    python tools/reset_bench.py [--envs 4096 65536] [--repeats 5]

Prints one JSON line per size: host-wall ms per reset (reset call + stream sync) for reference-RNG
resets after a stepped day (as SB3's automatic reset follows a day) and back to back, device-RNG and
replay resets, and the host threads used.
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

from smart_nanogrid_gym import SmartNanogridVecEnv  # noqa: E402
from smart_nanogrid_gym._native import lib  # noqa: E402


def timed(fn, repeats, sync=True, between=None):
    """Host-wall ms of fn(); between(), untimed, runs before each repetition.  sync=True waits for the
    whole device (work the call left on side streams included), "stream" for the caller's stream only (what
    the next step_tensors is ordered after), False for nothing (the host call alone)."""
    out = []
    for _ in range(repeats):
        if between is not None:
            between()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if sync == "stream":
            torch.cuda.current_stream().synchronize()
        elif sync:
            torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    return {"median_ms": float(np.median(out)), "min_ms": float(np.min(out)), "max_ms": float(np.max(out))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, nargs="+", default=[4096, 65536])
    ap.add_argument("--chargers", type=int, default=10)
    ap.add_argument("--repeats", type=int, default=9)
    args = ap.parse_args()
    kw = dict(number_of_chargers=args.chargers, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse")
    for E in args.envs:
        v = SmartNanogridVecEnv(E, seed=1, rng="reference", **kw)
        v.reset_tensors()   # first call: allocates streams and pinned staging
        zero = torch.zeros((E, v.act_dim), device=v.device)

        def day():   # the day a reset follows (SB3's automatic reset comes after the last step)
            for t in range(v.timesteps):
                v.step_tensors(zero)

        res = {"envs": E, "chargers": args.chargers, "host_threads": int(lib().sng_host_threads()),
               # after a stepped day: the next day's stream blocks were prepared while it was stepped
               "reference_reset": timed(lambda: v.reset_tensors(rng="reference"), args.repeats, between=day),
               # the same, until the observations are ready on the caller's stream (the next day's stream
               # blocks are still being prepared on the side stream, overlapping the day's steps)
               "reference_reset_stream_sync": timed(lambda: v.reset_tensors(rng="reference"), args.repeats,
                                                    sync="stream", between=day),
               # resets back to back: the preparation of each day's blocks waits on the critical path
               "reference_reset_back_to_back": timed(lambda: v.reset_tensors(rng="reference"), args.repeats),
               "device_reset": timed(lambda: v.reset_tensors(rng="device"), args.repeats)}
        # a whole reference-RNG day (reset + its steps), device-synced: the side-stream preparation
        # overlaps the steps
        res["reference_day"] = timed(lambda: (v.reset_tensors(rng="reference"), day()), args.repeats)
        res["device_day"] = timed(lambda: (v.reset_tensors(rng="device"), day()), args.repeats)
        v.reset_tensors(rng="reference")
        for t in range(v.timesteps):
            v.step_tensors(zero)
        res["replay_reset"] = timed(lambda: v.replay_tensors(), args.repeats)
        # the host part alone: the call returns once its work is queued (no stream sync)
        res["replay_call_only"] = timed(lambda: v.replay_tensors(), args.repeats, sync=False)
        res["reference_call_only"] = timed(lambda: v.reset_tensors(rng="reference"), args.repeats, sync=False)
        os.environ["SNG_HOST_THREADS"] = "1"
        res["replay_reset_1thread"] = timed(lambda: v.replay_tensors(), args.repeats)
        del os.environ["SNG_HOST_THREADS"]
        res["timeline_mb"] = round(v.timesteps * args.chargers * E * 12 / 1e6, 1)
        print(json.dumps(res), flush=True)
        v.close()


if __name__ == "__main__":
    main()
