"""Split a rocprofv3 kernel trace (`--kernel-trace --output-format csv`, *_kernel_trace.csv) of
`bench.py` into the step kernel's dispatches inside graph replays (back-to-back behind the previous
node) and the eager HIP-event probe days, and by timestep within the day.

    python tools/trace_split.py gpurun_out/prof [kernel-substring]
"""
import csv
import glob
import os
import sys

import numpy as np


def load(path_or_dir):
    files = [path_or_dir] if path_or_dir.endswith(".csv") else glob.glob(
        os.path.join(path_or_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fp:
            for r in csv.DictReader(fp):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main():
    rows = load(sys.argv[1])
    key = sys.argv[2] if len(sys.argv) > 2 else "step_"
    gen = "generate_kernel"
    prev_end = None
    t = -1
    cls = {"graph": [], "eager": []}
    by_t = {}
    for s, e, name in rows:
        if gen in name:
            t = 0
        elif key in name and "bump" not in name:
            gap = None if prev_end is None else (s - prev_end) / 1e3
            kind = "graph" if gap is not None and gap < 3.0 else "eager"
            d = (e - s) / 1e3
            cls[kind].append((d, gap))
            by_t.setdefault((kind, t), []).append(d)
            t += 1
        prev_end = e
    for k, v in cls.items():
        if not v:
            continue
        d = np.array([x[0] for x in v])
        g = np.array([x[1] for x in v if x[1] is not None])
        print(f"{k}: n={len(d)} mean={d.mean():.3f} us median={np.median(d):.3f} min={d.min():.3f} "
              f"max={d.max():.3f}  gap before mean={g.mean() if len(g) else float('nan'):.3f} us")
    for kind in ("graph", "eager"):
        ts = sorted(t for (k, t) in by_t if k == kind)
        if ts:
            print(kind, "by t:", " ".join(f"{t}:{np.mean(by_t[(kind, t)]):.2f}" for t in ts))


if __name__ == "__main__":
    main()
