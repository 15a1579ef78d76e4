"""Where a reference-RNG day's time goes, next to a device-RNG day's (65,536 x 10 by default): eager days of
reset_tensors + 24 step_tensors (zero actions, as tools/reset_bench.py), device-synced per day, reference days
then device days.  Run it under `rocprofv3 --kernel-trace` and split the trace with --split <kernel_trace.csv>:
per kernel name the dispatches and mean duration, per day kind the kernels' summed time.

    rocprofv3 --kernel-trace -d gpurun_out/refday -o run --output-format csv -- python tools/diag/refday_split.py
    python tools/diag/refday_split.py --split gpurun_out/refday/run_kernel_trace.csv
"""
import argparse
import csv
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))


def run(args):
    import numpy as np
    import torch

    from smart_nanogrid_gym import SmartNanogridVecEnv
    kw = dict(number_of_chargers=args.chargers, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse")
    v = SmartNanogridVecEnv(args.envs, seed=1, rng="reference", **kw)
    zero = torch.zeros((args.envs, v.act_dim), device=v.device)
    out = {}
    for kind in ("reference", "device"):
        walls = []
        for d in range(args.warmup + args.days):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            v.reset_tensors(rng=kind)
            for t in range(v.timesteps):
                v.step_tensors(zero)
            torch.cuda.synchronize()
            if d >= args.warmup:
                walls.append((time.perf_counter() - t0) * 1e3)
        out[kind + "_day_ms"] = round(float(np.median(walls)), 4)
        time.sleep(0.05)   # a gap in the trace between the two kinds
    print(json.dumps(out), flush=True)
    v.close()


def split(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the two kinds are separated by the 50 ms sleep
    phases, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > 20_000_000:
            phases.append(cur)
            cur = []
        cur.append((r["Kernel_Name"], s, e))
        last_end = max(e, last_end or e)
    phases.append(cur)
    for i, ph in enumerate(phases):
        by = {}
        for name, s, e in ph:
            short = name.split("(")[0]
            by.setdefault(short, []).append((e - s) / 1e3)
        span = (max(e for _, _, e in ph) - min(s for _, s, _ in ph)) / 1e3
        print(f"phase {i}: {len(ph)} dispatches over {span:.1f} us")
        for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            print(f"   {len(v):5d} x {sum(v) / len(v):8.2f} us  {k}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--chargers", type=int, default=10)
    ap.add_argument("--days", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--split", help="split a rocprofv3 kernel trace instead of running")
    args = ap.parse_args()
    if args.split:
        split(args.split)
    else:
        run(args)


if __name__ == "__main__":
    main()
