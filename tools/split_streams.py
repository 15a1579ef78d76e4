"""Experiment: the bench day (65,536 envs x 10 chargers) as S independent env slices, each a
hipGraph of D days replayed on its own HIP stream, so one slice's compute phase overlaps another's
memory phase.  Prints ms/day and env-steps/s per S.

    python tools/split_streams.py [S ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))

import torch  # noqa: E402

from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv  # noqa: E402


def run(S, E=65536, N=10, days=5, warm=2, D=20):
    kw = dict(number_of_chargers=N, time_interval="1h", charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse", pv_system_available_in_model=True,
              battery_system_available_in_model=True)
    dev = torch.device("cuda", 0)
    per = E // S
    venvs, graphs, streams = [], [], []
    for k in range(S):
        v = SmartNanogridVecEnv(per, seed=2024, device=0, rng="device", env_offset=k * per, **kw)
        g = torch.Generator(device=dev).manual_seed(k)
        low = torch.tensor(v.action_space.low, device=dev)
        high = torch.tensor(v.action_space.high, device=dev)
        acts = (low + (high - low) * torch.rand((v.timesteps, per, v.act_dim), generator=g, device=dev)).contiguous()
        v._info.flags = None
        venvs.append(v)
        graphs.append(EpisodeGraph(v, acts, with_reset=True, days=D))
        streams.append(torch.cuda.Stream(dev))
    def day():
        for g, s in zip(graphs, streams):
            g.launch(s.cuda_stream)
    for _ in range(warm):
        day()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(days):
        day()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (days * D)
    print(f"S={S}: {dt * 1e3:.4f} ms/day  {E * 24 / dt:.4e} env-steps/s", flush=True)
    for g in graphs:
        g.close()
    for v in venvs:
        v.close()


if __name__ == "__main__":
    for S in [int(x) for x in sys.argv[1:]] or [1, 2, 4]:
        run(S)
