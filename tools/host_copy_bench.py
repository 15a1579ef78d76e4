"""Host-side copy of one step's observations out of the pinned staging buffer (the SB3 path returns fresh
numpy arrays every step): numpy's copy against torch's multi-threaded CPU copy into a fresh array, and the
terminal_observation infos of a done step.  65,536 x 29 float32 = 7.6 MB.

    python tools/host_copy_bench.py [--envs 65536] [--reps 50]
"""
import argparse
import itertools
import json
import time

import numpy as np
import torch


def med(fn, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return round(float(np.median(ts)) * 1e3, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--obs", type=int, default=29)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    E, O = args.envs, args.obs
    src = torch.rand((E, O), dtype=torch.float32)
    src = src.pin_memory() if torch.cuda.is_available() else src   # the staging buffer is pinned on the GPU box
    srcn = src.numpy()

    def torch_copy():
        out = np.empty((E, O), np.float32)
        torch.from_numpy(out).copy_(src)
        return out

    obs = srcn.copy()
    res = {"envs": E, "bytes": E * O * 4, "torch_threads": torch.get_num_threads(),
           "numpy_copy_ms": med(lambda: srcn.copy(), args.reps),
           "torch_copy_ms": med(torch_copy, args.reps),
           "terminal_infos_ms": med(lambda: [{"terminal_observation": o, "TimeLimit.truncated": False} for o in obs],
                                    max(5, args.reps // 5)),
           "terminal_infos_zip_ms": med(lambda: list(map(dict, zip(zip(itertools.repeat("terminal_observation"), obs),
                                                                   itertools.repeat(("TimeLimit.truncated", False))))),
                                        max(5, args.reps // 5)),
           "rows_list_ms": med(lambda: list(obs), max(5, args.reps // 5)),
           "rows_unbind_ms": med(lambda: torch.from_numpy(obs).unbind(0), max(5, args.reps // 5)),
           "empty_infos_ms": med(lambda: list(itertools.starmap(dict, itertools.repeat((), E))), max(5, args.reps // 5))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
