"""Where a reference-RNG day's wavefront spends its time (ref_day2_kernel, diagnostic build with stamps).

    make -C tools/diag stamps
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_stamps.so python tools/rd_stamps.py [--envs 65536]

Per wavefront (64 envs): stamp 0 its start, stamp 1 its end, and the s_memrealtime ticks (10 ns) spent in
phase 1 (the vehicles' draws, ring refills included) and phase 2 (the timeline walk and its stores) summed
over the chargers.  The stamps take no wait of their own, so a wait for earlier stores shows up where the
program next waits on memory (a refill of the next charger's phase 1).
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smart_nanogrid_gym import SmartNanogridVecEnv, _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--days", type=int, default=6)
    args = ap.parse_args()
    L = _native.lib()
    setter = L.sng_debug_set_stamps
    setter.argtypes = [ctypes.c_void_p]
    E = args.envs
    venv = SmartNanogridVecEnv(E, seed=5, rng="reference", number_of_chargers=10, time_interval="1h",
                               charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    blocks = (E + 63) // 64
    buf = torch.zeros(max(blocks, 4096) * 8, dtype=torch.int64, device=venv.device)
    acts = torch.rand((24, E, venv.act_dim), device=venv.device)
    rows = []
    for day in range(args.days):
        torch.cuda.synchronize()
        buf.zero_()
        assert setter(ctypes.c_void_p(buf.data_ptr())) == 0
        venv.reset_tensors()
        torch.cuda.synchronize()
        assert setter(ctypes.c_void_p(0)) == 0
        if day > 0:
            rows.append(buf.view(-1, 8)[:blocks, :4].cpu().numpy().astype(np.float64) * 10.0)   # ns
        for t in range(24):
            venv.step_tensors(acts[t])
    venv.close()
    st = np.stack(rows)   # [days, waves, 4]
    span = st[..., 1].max(axis=1) - st[..., 0].min(axis=1)
    own = st[..., 1] - st[..., 0]
    q = lambda x: f"med {np.median(x) / 1e3:7.2f}  p10 {np.percentile(x, 10) / 1e3:7.2f}  p90 {np.percentile(x, 90) / 1e3:7.2f} us"
    print(f"ref_day2_kernel, {E} envs, {blocks} wavefronts, {args.days - 1} days")
    print("kernel span (first start to last end) ", q(span))
    print("wavefront start (rel. first)         ", q(st[..., 0] - st[..., 0].min(axis=1, keepdims=True)))
    print("wavefront own time                   ", q(own))
    print("  phase 1 (draws, refills)           ", q(st[..., 2]))
    print("  phase 2 (timeline walk, stores)    ", q(st[..., 3]))
    print("  rest (setup, position store)       ", q(own - st[..., 2] - st[..., 3]))


if __name__ == "__main__":
    main()
