"""Per-workgroup phase timeline of the step kernel (diagnostic build libsng_stamps.so, tools/diag).

    make -C tools/diag stamps
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_stamps.so python tools/stamps.py [lanes]

lanes 0 (default) times the headline's kernel (step_wide_kernel, two lanes per env, 32 envs per
one-wavefront workgroup); lanes 1 the lean kernel (64 envs per workgroup).  The stamps add no wait of
their own (s_memrealtime, 100 MHz, when the workgroup's wavefront reaches the point): 0 = start,
1 = actions tile staged (the tile and the per-env values landed), 2 = chargers done, 3 = env tail done
(observation tile complete), 4 = observation stores issued.  The
kernel's device time per step comes from the HIP-event probe of the same process, so the stretch after
stamp 4 (store drain + end of kernel) is that time minus the last stamp.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smart_nanogrid_gym import SmartNanogridVecEnv, _native  # noqa: E402


def main():
    L = _native.lib()
    setter = getattr(L, "sng_debug_set_stamps")
    setter.argtypes = [ctypes.c_void_p]
    E, N = int(os.environ.get("ENVS", 65536)), 10
    v2x = "--v2x" in sys.argv   # a V2X station: the lean kernel, Box actions in [-1, 1]
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lanes = int(args[0]) if args else 0
    venv = SmartNanogridVecEnv(E, seed=3, rng="device", number_of_chargers=N, time_interval="1h",
                               charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse",
                               step_lanes_per_env=lanes, vehicle_to_everything=v2x)
    print("kernel:", venv.step_kernel_name())
    venv.reset_tensors()
    print("stepped by:", venv.step_kernel_name())
    per_block = 32 if "step_wide_kernel" in venv.step_kernel_name() else 64
    blocks = (E + per_block - 1) // per_block   # one wavefront per workgroup; 8 stamp slots per block
    buf = torch.zeros(blocks * 8, dtype=torch.int64, device="cuda:0")
    assert setter(ctypes.c_void_p(buf.data_ptr())) == 0
    g = torch.Generator(device="cuda:0").manual_seed(1)
    acts = torch.rand((24, E, N + 1), device="cuda:0", generator=g)
    acts[..., -1] = acts[..., -1] * 2 - 1
    if v2x:
        acts = acts * 2 - 1
    acts = torch.where(torch.rand(acts.shape, device="cuda:0", generator=g) < 0.2, torch.zeros_like(acts), acts)
    rows, ts, ids = [], [], []
    for day in range(3):
        venv.reset_tensors()
        for t in range(24):
            venv.step_tensors(acts[t])
            torch.cuda.synchronize()
            if day > 0:
                b = buf.view(blocks, 8).cpu().numpy()
                rows.append(b[:, :5].astype(np.float64) * 10.0)   # ns
                ids.append(b[:, 6:8])
                ts.append(t)
    allph = np.stack(rows)                      # [steps, blocks, 5]
    allph = allph - allph[..., :1].min(axis=1, keepdims=True)
    ts = np.array(ts)
    for label, sel in (("eager t = 0", ts == 0), ("eager t >= 1", ts > 0)):
        print(f"--- {label}")
        report(allph[sel], np.stack(ids)[sel])
    ms = venv.time_step_kernels(acts, days=1)
    print(f"HIP-event step time: t = 0 {ms[0] * 1e3:.3f} us, t >= 1 mean {np.mean(ms[1:]) * 1e3:.3f} us")
    # in a day graph (as the bench runs it): the stamps of the day's last step, t = T - 1
    from smart_nanogrid_gym import EpisodeGraph
    gr = EpisodeGraph(venv, acts.contiguous(), with_reset=True, days=1)
    rows, ids = [], []
    for rep in range(6):
        gr.launch()
        torch.cuda.synchronize()
        if rep > 0:
            b = buf.view(blocks, 8).cpu().numpy()
            rows.append(b[:, :5].astype(np.float64) * 10.0)
            ids.append(b[:, 6:8])
    gr.close()
    allph = np.stack(rows)
    allph = allph - allph[..., :1].min(axis=1, keepdims=True)
    print("--- graph, t = 23")
    report(allph, np.stack(ids))
    setter(ctypes.c_void_p(0))
    venv.close()


def report(ph, ids):
    q = lambda x: f"med {np.median(x) / 1e3:6.3f}  p10 {np.percentile(x, 10) / 1e3:6.3f}  p90 {np.percentile(x, 90) / 1e3:6.3f} us"
    names = ["start (rel. first WG)", "tile + per-env landed", "chargers", "env tail", "obs stores issued"]
    print(f"{'wave start':28s}", q(ph[..., 0]))
    for k in range(1, 5):
        print(f"{names[k]:28s}", q(ph[..., k] - ph[..., k - 1]))
    print(f"{'last WG reaches stamp 4':28s}", q(ph[..., 4].max(axis=1)))
    st = ph[..., 0]
    print("wave start deciles (us):", " ".join(f"{np.percentile(st, p) / 1e3:.2f}" for p in range(0, 101, 10)))
    xcc = ids[..., 0] & 0xf
    print("per XCC: median start / median stamp 4 (us):",
          " ".join(f"{x}:{np.median(st[xcc == x]) / 1e3:.2f}/{np.median(ph[..., 4][xcc == x]) / 1e3:.2f}"
                   for x in range(8) if (xcc == x).any()))
    # waves sharing a SIMD (HW_ID: SIMD bits 5:4, CU 11:8, SH 12, SE 15:13; with the XCC id), last sample
    hw = ids[-1].astype(np.int64)
    key = ((hw[:, 0] & 0xf) << 16) | (hw[:, 1] & 0xff30)
    _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    per = cnt[inv]
    print("waves per SIMD (last sample): " + ", ".join(
        f"{k}: {np.sum(per == k)} waves, median stamp 4 {np.median(ph[-1, per == k, 4]) / 1e3:.2f} us, "
        f"max {ph[-1, per == k, 4].max() / 1e3:.2f} us" for k in sorted(set(per.tolist()))))
    # block index order vs start: dispatch order
    nb = st.shape[-1]
    for part in range(4):
        sl = slice(part * nb // 4, (part + 1) * nb // 4)
        print(f"  blocks {sl.start}-{sl.stop - 1}: median start {np.median(st[..., sl]) / 1e3:.2f} us")


if __name__ == "__main__":
    main()
