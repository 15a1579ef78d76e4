"""Per-wave time split of the reference-RNG day kernel (diagnostic build libsng_rdprof.so, -DSNG_RD2_PROF).

    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_rdprof.so python tools/rd_prof.py [envs...]

Per wavefront (64 envs): kernel span (s_memrealtime, 100 MHz), shader-clock cycles in phase 1 (draws),
phase 2 (timeline stores, drained), in ring refills (drained), refill count, phase-1 iterations (the
busiest lane's draw steps summed over chargers) and dry-ring direct loads.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smart_nanogrid_gym import SmartNanogridVecEnv, _native  # noqa: E402


def main():
    L = _native.lib()
    setter = L.sng_debug_set_stamps
    setter.argtypes = [ctypes.c_void_p]
    for E in [int(x) for x in sys.argv[1:]] or [4096, 65536]:
        venv = SmartNanogridVecEnv(E, seed=3, rng="reference", number_of_chargers=10, time_interval="1h",
                                   charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
        waves = (E + 63) // 64
        buf = torch.zeros(waves * 8, dtype=torch.int64, device="cuda:0")
        assert setter(ctypes.c_void_p(buf.data_ptr())) == 0
        rows = []
        for day in range(4):
            buf.zero_()
            venv.reset_tensors()
            torch.cuda.synchronize()
            rows.append(buf.view(waves, 8).cpu().numpy().astype(np.float64))
        setter(ctypes.c_void_p(0))
        r = np.concatenate(rows[1:])
        span_us = (r[:, 1] - r[:, 0]) / 100.0
        cyc = lambda k: float(np.median(r[:, k]))   # noqa: E731
        print(json.dumps({"envs": E, "waves": waves, "span_us_median": float(np.median(span_us)),
                          "span_us_max": float(span_us.max()), "phase1_cycles": cyc(2), "phase2_cycles": cyc(3),
                          "refill_cycles": cyc(4), "refills": cyc(5), "phase1_iterations": cyc(6),
                          "dry_loads": cyc(7)}))
        venv.close()


if __name__ == "__main__":
    main()
