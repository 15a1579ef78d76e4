"""A/B equality of two builds' device-RNG days: for each station, penalty mode and size, the SHA-256 of the
whole handle state after a device reset (sng_get_state: the record timeline, SoC seed, PV ratio ...) and of the
observations and rewards of the day stepped with fixed actions.  Run once per library and diff the lines:

    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_<old>.so python tools/diag/gen_ab_check.py > a.txt
    python tools/diag/gen_ab_check.py > b.txt && diff a.txt b.txt

A generator rewrite that keeps the same draws (round 6's gen_walk_masks) must print the same lines.
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smart_nanogrid_gym import SmartNanogridVecEnv  # noqa: E402


def main():
    cases = [(4096, 10, m, "1h") for m in ("sparse", "dense", "on_departure", "no_penalty")]
    cases += [(4096, n, "sparse", "1h") for n in (1, 4, 7, 16, 33)]
    cases += [(65536, 10, "sparse", "1h"), (1000, 10, "dense", "2h"), (512, 10, "sparse", "30min")]
    # stations above 60 chargers (round 6: the same one launch), stochastic profiles (config 5's day), requested SoC
    cases += [(2048, 64, "sparse", "1h"), (1024, 128, "dense", "1h"), (4096, 50, "sparse", "15min", "noise"),
              (4096, 10, "sparse", "1h", "req"), (300, 12, "on_departure", "30min", "noise")]
    for E, N, mode, ti, *extra in cases:
        kw = dict(number_of_chargers=N, time_interval=ti, charging_mode="bounded", vehicle_uncharged_penalty_mode=mode)
        if ti.endswith("min"):   # below 1 h the day needs the build-defined extension (sng_create refuses it)
            kw.update(extended_day=True)
        if "noise" in extra:
            kw.update(extended_day=True, pv_noise=0.2, price_noise=0.1)
        if "req" in extra:
            kw.update(enable_requested_state_of_charge=True)
        v = SmartNanogridVecEnv(E, seed=97, rng="device", **kw)
        g = torch.Generator(device="cuda:0").manual_seed(5)
        acts = torch.rand((v.timesteps, E, v.act_dim), device="cuda:0", generator=g)
        acts[..., -1] = acts[..., -1] * 2 - 1
        for day in range(2):
            obs0 = v.reset_tensors().clone()
            h_state = hashlib.sha256(v.save_state()).hexdigest()[:16]
            h = hashlib.sha256(obs0.cpu().numpy().tobytes())
            for t in range(v.timesteps):
                o, r, _ = v.step_tensors(acts[t])
                h.update(o.cpu().numpy().tobytes())
                h.update(r.cpu().numpy().tobytes())
            print(f"E={E} N={N} {mode} {ti} {'+'.join(extra)} day{day}: state {h_state} day {h.hexdigest()[:16]}")
        v.close()


if __name__ == "__main__":
    main()
