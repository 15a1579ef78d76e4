"""Host cost of replaying the bench's day graphs (hipGraphLaunch of 20 days = 500 kernel nodes).

The bench's wall clock per day (ms_per_step) matched the HIP-event device time per day in rounds 2-4
(0.168-0.172 ms).  A round-5 box measured 0.252 ms wall against 0.1675 ms device time: the host did not
keep the GPU fed.  This probe measures, per HIP runtime setting (each in a fresh child process):
  launch_ms  host time of one sng_graph_launch call (perf_counter around it), median over the replays;
  wall_ms    wall time per day over R back-to-back replays (synchronised at both ends);
  gpu_ms     HIP-event device time per day over the same replays.

    python tools/launch_cost.py [--days 20] [--replays 10] [--envs 65536]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = [
    {},
    {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "1"},
    {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "0"},
    {"DEBUG_HIP_GRAPH_BATCH_SIZE": "1000"},
    {"HIP_FORCE_DEV_KERNARG": "1"},
]


def child(args):
    sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))
    import numpy as np
    import torch
    from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv
    E = args.envs
    venv = SmartNanogridVecEnv(E, seed=7, device=0, rng="device", number_of_chargers=10, time_interval="1h",
                               charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
    T, A = venv.timesteps, venv.act_dim
    acts = torch.rand((T, E, A), device=venv.device)
    venv.reset_tensors(rng="device")
    g = EpisodeGraph(venv, acts, with_reset=True, days=args.days)
    for _ in range(3):
        g.launch()
    torch.cuda.synchronize()
    launch = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.replays):
        a = time.perf_counter()
        g.launch()
        launch.append(time.perf_counter() - a)
    ev1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # launches with the GPU idle before each (synchronised): the host cost alone
    idle = []
    for _ in range(5):
        torch.cuda.synchronize()
        a = time.perf_counter()
        g.launch()
        idle.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    days = args.days * args.replays
    out = {"env": {k: v for k, v in os.environ.items() if k in {x for d in VARIANTS for x in d}},
           "launch_ms": float(np.median(launch)) * 1e3, "launch_ms_max": max(launch) * 1e3,
           "launch_idle_ms": float(np.median(idle)) * 1e3,
           "wall_ms_per_day": wall / days * 1e3, "gpu_ms_per_day": ev0.elapsed_time(ev1) / days,
           "nodes_per_launch": args.days * (T + 1)}
    g.close()
    venv.close()
    print("RESULT " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=int, default=20)
    ap.add_argument("--replays", type=int, default=10)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        return child(args)
    for v in VARIANTS:
        env = dict(os.environ, **v)
        r = subprocess.run([sys.executable, __file__, "--child", "--days", str(args.days), "--replays",
                            str(args.replays), "--envs", str(args.envs)], env=env, capture_output=True, text=True,
                           timeout=300)
        line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
        print(json.dumps(v), line[0][7:] if line else f"rc={r.returncode} {r.stderr[-500:]}", flush=True)
        if r.returncode != 0:
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
