"""Where a reference-RNG day's wavefront spends its time (ref_day2_kernel, diagnostic build with stamps).

    make -C tools/diag stamps
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_stamps.so python tools/rd_stamps.py [--envs 65536]

Per workgroup (64 envs, two wavefronts since round 5): stamp 0 its start, 1 the drawing wavefront's end,
4 the timeline wavefront's end, and the s_memrealtime ticks (10 ns) the drawing wavefront spent in phase 1
(the vehicles' draws, ring refills included, 2) and the timeline wavefront in phase 2 (the walk and its
stores, 3), summed over the chargers; 7 and 5 the two wavefronts' HW_ID (CU, SIMD, wave slot), so the table
shows how often both sit on one SIMD and how often two drawing wavefronts share one.  The stamps take no
wait of their own.
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
    rows, ids = [], []
    for day in range(args.days):
        torch.cuda.synchronize()
        buf.zero_()
        assert setter(ctypes.c_void_p(buf.data_ptr())) == 0
        venv.reset_tensors()
        torch.cuda.synchronize()
        assert setter(ctypes.c_void_p(0)) == 0
        if day > 0:
            raw = buf.view(-1, 8)[:blocks].cpu().numpy()
            rows.append(raw[:, :5].astype(np.float64) * 10.0)   # ns
            ids.append(raw[:, [6, 7, 5]])
        for t in range(24):
            venv.step_tensors(acts[t])
    venv.close()
    st = np.stack(rows)   # [days, workgroups, 6]
    end = np.maximum(st[..., 1], st[..., 4])
    span = end.max(axis=1) - st[..., 0].min(axis=1)
    own = end - st[..., 0]
    q = lambda x: f"med {np.median(x) / 1e3:7.2f}  p10 {np.percentile(x, 10) / 1e3:7.2f}  p90 {np.percentile(x, 90) / 1e3:7.2f} us"
    print(f"ref_day2_kernel, {E} envs, {blocks} workgroups, {args.days - 1} days")
    print("kernel span (first start to last end) ", q(span))
    print("workgroup start (rel. first)         ", q(st[..., 0] - st[..., 0].min(axis=1, keepdims=True)))
    print("workgroup own time                   ", q(own))
    print("  drawing wavefront: phase 1 (draws, refills)   ", q(st[..., 2]))
    print("  timeline wavefront: phase 2 (walk, stores)    ", q(st[..., 3]))
    print("  timeline wavefront ends after the drawing one ", q(st[..., 4] - st[..., 1]))
    # HW_ID (gfx9): wave slot bits 3:0, SIMD 5:4, CU 11:8, SH 12, SE 15:13; with the XCC id a SIMD's key
    hw = ids[-1].astype(np.int64)
    dkey = (hw[:, 0] << 16) | (hw[:, 1] & 0xff30)            # drawing wavefront: XCC, SE/SH/CU, SIMD
    wkey = ((hw[:, 2] >> 32) << 16) | (hw[:, 2] & 0xff30)    # timeline wavefront
    keys, counts = np.unique(dkey, return_counts=True)
    drawers = dict(zip(keys.tolist(), counts.tolist()))
    writers = dict(zip(*[a.tolist() for a in np.unique(wkey, return_counts=True)]))
    own_last = own[-1]
    print(f"last day: both wavefronts of a workgroup on one SIMD {np.mean(dkey == wkey):.1%}")
    for nd in sorted(set(drawers.values())):
        for nw in sorted(set(writers.values()) | {0}):
            m = np.array([drawers[int(k)] == nd and writers.get(int(k), 0) == nw for k in dkey])
            if m.any():
                print(f"  drawing wavefronts on a SIMD with {nd} drawing and {nw} timeline wavefronts: "
                      f"{m.sum():4d} workgroups, own time med {np.median(own_last[m]) / 1e3:6.2f} "
                      f"max {own_last[m].max() / 1e3:6.2f} us")


if __name__ == "__main__":
    main()
