"""The first steps after a device reset: per-timestep step-kernel time when the steps-only day graph starts right
after the reset (B) or after the GPU idled 2 ms (A).  If A's first steps are as fast as the rest, what slows them
is work the reset left behind (e.g. its output still being written back), not the data they read.

    rocprofv3 --kernel-trace -d gpurun_out/t0p -o run --output-format csv -- python tools/diag/t0_probe.py
    python tools/diag/t0_probe.py --split gpurun_out/t0p/run_kernel_trace.csv
"""
import argparse
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))


def run(reps):
    import torch

    from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv
    kw = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    v = SmartNanogridVecEnv(65536, seed=3, rng="device", **kw)
    g = torch.Generator(device="cuda:0").manual_seed(1)
    acts = torch.rand((24, 65536, v.act_dim), device="cuda:0", generator=g)
    acts[..., -1] = acts[..., -1] * 2 - 1
    v.reset_tensors()
    day = EpisodeGraph(v, acts, with_reset=False)
    for phase, idle in (("B", 0.0), ("A", 0.002)):
        for _ in range(reps):
            v.reset_tensors()
            if idle:
                torch.cuda.synchronize()
                time.sleep(idle)
            day.launch()
            torch.cuda.synchronize()
        time.sleep(0.05)   # a gap in the trace between the phases
    day.close()
    v.close()


def split(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur, last = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last is not None and s - last > 20_000_000:
            phases.append(cur)
            cur = []
        cur.append((r["Kernel_Name"], s, e))
        last = max(e, last or e)
    phases.append(cur)
    for ph in phases[-2:]:
        per_t, t = {}, None
        for name, s, e in ph:
            if "generate_kernel" in name:
                t = 0
            elif "step_wide_kernel" in name and t is not None:
                per_t.setdefault(t, []).append((e - s) / 1e3)
                t += 1
        if per_t:
            print(" ".join(f"{k}:{sum(v) / len(v):.2f}" for k, v in sorted(per_t.items())))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--split")
    a = ap.parse_args()
    if a.split:
        split(a.split)
    else:
        run(a.reps)


if __name__ == "__main__":
    main()
