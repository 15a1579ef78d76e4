import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "smart-nanogrid-gym_amd"))
import numpy as np, torch
from smart_nanogrid_gym import SmartNanogridVecEnv
KW = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse",
          pv_system_available_in_model=True, battery_system_available_in_model=True)
for E in (4096, 65536):
    v = SmartNanogridVecEnv(E, seed=2024, rng="device", **KW)
    v._info.flags = None
    rng = np.random.default_rng(1)
    v.reset_tensors()
    s0 = v.vehicle_state_of_charge()
    print(E, v.step_kernel_name(), "reset soc range", s0.min(), s0.max(), flush=True)
    for t in range(4):
        a = rng.uniform(0, 1, (E, 11)).astype(np.float32)
        o, r, d = v.step_tensors(torch.from_numpy(a).cuda())
        torch.cuda.synchronize()
        s = v.vehicle_state_of_charge()
        bad = np.argwhere(~((s >= 0) & (s <= 1)))
        ob = o.cpu().numpy()
        badobs = np.argwhere(~np.isfinite(ob) | (np.abs(ob) > 10))
        print(E, "t", t, "bad soc", len(bad), bad[:8].tolist(), "bad obs", len(badobs), badobs[:8].tolist(), flush=True)
        if len(bad):
            e = bad[0][0]
            print("  env", e, "soc", s[e].tolist(), "e%32", e % 32, "e//32", e // 32, flush=True)
            envs = np.unique(bad[:, 0]); print("  bad envs (first 40)", envs[:40].tolist(), "count", len(envs), flush=True)
            print("  chargers hist", np.bincount(bad[:, 1], minlength=10).tolist(), flush=True)
    v.close()
