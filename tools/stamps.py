"""Per-wave phase timeline of the step kernel (diagnostic build libsng_stamps.so).

    make -C smart-nanogrid-gym_amd/csrc stamps
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_stamps.so python tools/stamps.py [lanes...]

Stamps (s_memrealtime, 100 MHz) per workgroup: 0 = loads issued, 1 = actions staged and all
loads landed (forced wait), 2 = env computed (obs in LDS), 3 = obs stored and drained.
Prints, per lanes setting, the median/p90 of each phase and the spread of wave start times.
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
    lanes_list = [int(x) for x in sys.argv[1:]] or [1, 2]
    L = _native.lib()
    setter = getattr(L, "sng_debug_set_stamps")
    setter.argtypes = [ctypes.c_void_p]
    E, N = 65536, 10
    for lanes in lanes_list:
        venv = SmartNanogridVecEnv(E, seed=3, rng="device", step_lanes_per_env=lanes, number_of_chargers=N,
                                   time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
        blocks = (E * lanes + 255) // 256   # 256-thread workgroups, 256 / lanes envs each
        buf = torch.zeros(blocks * 4, dtype=torch.int64, device="cuda:0")
        assert setter(ctypes.c_void_p(buf.data_ptr())) == 0
        acts = torch.rand((24, E, N + 1), device="cuda:0")
        acts[..., -1] = acts[..., -1] * 2 - 1
        phases = []
        for day in range(2):
            venv.reset_tensors()
            for t in range(24):
                venv.step_tensors(acts[t])
                torch.cuda.synchronize()
                s = buf.view(blocks, 4).cpu().numpy().astype(np.float64) * 10.0   # ns
                if day == 1:
                    phases.append(s - s[:, :1].min())
        ph = np.stack(phases)   # [24, blocks, 4]
        start, land, comp, end = ph[..., 0], ph[..., 1], ph[..., 2], ph[..., 3]
        q = lambda x: f"med {np.median(x) / 1e3:6.2f} p90 {np.percentile(x, 90) / 1e3:6.2f} us"
        print(f"lanes={lanes} waves={blocks}")
        print("  wave start (rel. first) ", q(start))
        print("  loads landed            ", q(land - start))
        print("  compute                 ", q(comp - land))
        print("  obs store + drain       ", q(end - comp))
        print("  last wave end (kernel)  ", q(end.max(axis=1)))
        setter(ctypes.c_void_p(0))
        venv.close()


if __name__ == "__main__":
    main()
