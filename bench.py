"""Throughput of the batched SmartNanogridEnv hot path on MI355X.

Metric (BASELINE.json): env-steps/sec (whole node) at 65,536 envs x 10 chargers, 24-step day.
One bench "step" = one simulated day for every env on every GPU: GPU-RNG reset (new
vehicles) + 24 fused step kernels, replayed as hipGraphs of 20 days.  When N > 1 every day's
per-env returns are all-gathered over RCCL, one collective per replay on the collective
stream, overlapped with the next replay's kernels.  Actions are synthetic (uniform in the
action Box, 20 % exact zeros), pre-generated on the device outside the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--chargers C] [--no-cpu-baseline]
        # N > 1: this process measures cpu_baseline, then starts N rank processes itself
        # (torch.distributed.run as a child process) and exits with their status
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
        [--dist-backend gloo]   # several ranks on one GPU: day returns gathered through host memory
    A launcher's WORLD_SIZE that differs from --gpus is refused (exit 2), as is --gpus N > 1 with RCCL
    and fewer than N visible GPUs.  The line's `dist` object reports the process group's backend and the
    world size it initialised.

Rank 0 prints one JSON line.  `roofline` describes the dominant kernel (the fused step):
achieved = SURVEY.md 8(d)'s algorithmic bytes per env-step, B(N) = 40 N + 65 (465 B at N = 10),
x the envs of one launch / the step kernel's mean duration inside the day graphs: the HIP-event device
time of a timed day (on the graphs' stream) less the reset kernel, over the T step dispatches -- the
start-to-start time rocprofv3 reports for a graph's kernels.  The reset kernel's time and the isolated
dispatch time of the step kernel (`eager_launch_us`, `frac_eager`) come from HIP start/stop events
attached to every dispatch of eager days right after the timed region, on the stream the kernels run on.
`frac_rocprof` is the same bytes over the average duration of that kernel in the committed
rocprofv3 --kernel-trace --stats summary (profiles/) of this very build (`build_id`, sng_build_id(): the
SHA-256 of the library's sources), null when none is committed for it.  Beside the
SURVEY.md 8(d) fraction: `frac_layout` prices the bytes this layout actually moves (32N + 89 B per env-step;
+4 B with --per-env-flags), `frac_pmc` the PMC-measured HBM bytes (`traffic`,
from the committed passes, null if absent), and `copy_step_size` / `copy_1gib` are the measured ceiling
SURVEY.md 8(d) asks for: libsng's float4 copy probe (sng_bandwidth_probe) moving the step's own read and
write bytes in one dispatch, and 1 GiB.  The step is timed with the default SngInfo of
SmartNanogridVecEnv: the day return and the flag summary word (touched only when an env raises a flag);
--per-env-flags adds the per-step per-env flag store the diagnostics use.  `cpu_baseline` is the C restatement of the reference's step()/reset()
(oracle/, kind "port", label "restatement") run as one process per host core granted by the cgroup CPU
quota (sched_getaffinity shows the whole machine on a GPU box), measured before the GPU is touched, with
the reference's own Python step() range from SURVEY.md section 6 beside it.
"""
import argparse
import json
import multiprocessing
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "smart-nanogrid-gym_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "env-steps/sec (whole node) at N=65,536 envs × 10 chargers, 24-step day"


def survey_bytes(n):
    """SURVEY.md 8(d) canonical algorithmic bytes per env-step (b-pv): actions 4(N+1) + obs 4(2N+9) +
    reward 8 + done 1 + EV SoC r/w 16N + BESS r/w 16 + scenario 12N = 40 N + 65."""
    return 40 * n + 65


def step_kernel_bytes(n, noise=False, flags=False):
    """What this layout moves per env-step of a device-RNG day (b-pv, no requested-SoC stream), as
    (read, written): reads = actions 4(N+1) + packed 2-byte charger-step record 2N (round 4; sng_layout.h)
    + EV SoC 8N + BESS 8 + PV ratio 8 + day return 8 (+ 8 for the env's two stochastic-profile keys);
    writes = obs 4(2N+9) + reward 8 + done 1 + EV SoC 8N + BESS 8 + day return 8 (+ 4 for the per-env
    per-step error flags, flags=True: the diagnostics' SngInfo.flags; the default SngInfo watches the
    one-word flag summary instead).  30N + 89 (+4) in all.  Host-RNG days read the word and a float64
    static SoC instead: 40N + 89."""
    rd = 4 * (n + 1) + 2 * n + 8 * n + 8 + 8 + 8 + (8 if noise else 0)
    wr = 4 * (2 * n + 9) + 8 + 1 + 8 * n + 8 + 8 + (4 if flags else 0)
    return rd, wr


def _cpu_worker(job):
    """One host process of the CPU baseline: whole days (reset + T steps) of independent oracle envs."""
    kw, budget_s, wid = job
    import oracle as O
    cfg = O.OracleConfig(**kw)
    batch = 256
    rng = np.random.default_rng(wid)
    acts = rng.uniform(0, 1, (cfg.T, batch, cfg.act_dim)).astype(np.float32)
    acts[..., -1] = acts[..., -1] * 2 - 1
    acts[rng.random(acts.shape) < 0.2] = 0
    envs = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        O.run_batch(cfg, batch, 10_000_000 * wid + envs, 1, acts)
        envs += batch
    return envs * cfg.T, time.perf_counter() - t0


def cgroup_cpus():
    """The CPU share the cgroup grants this process: cpu.max (cgroup v2) or cfs_quota_us / cfs_period_us
    (v1) as (cores, text); (None, text) when there is no quota."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as fp:
                txt = fp.read().strip()
        except OSError:
            continue
        if parse is not None:
            quota, period = parse(txt)[:2]
        else:
            try:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fp:
                    period = fp.read().strip()
            except OSError:
                return None, f"{path}={txt}"
            quota = txt
        src = f"{path}={txt}" + ("" if parse is not None else f"/{period}")
        if quota in ("max", "-1"):
            return None, src
        return max(1, int(int(quota) // int(period))), src
    return None, "no cgroup cpu quota file"


def cpu_baseline(kw, budget_s):
    """The restatement on every host core this process is granted, one process per core, forked before
    the GPU is initialised: the cgroup CPU quota (a GPU box shows the whole machine in sched_getaffinity
    but grants a share of it), else sched_getaffinity capped by OMP_NUM_THREADS; SNG_CPU_BASELINE_PROCS
    overrides both."""
    affinity = len(os.sched_getaffinity(0))
    quota, quota_src = cgroup_cpus()
    omp = os.environ.get("OMP_NUM_THREADS")
    forced = os.environ.get("SNG_CPU_BASELINE_PROCS")
    if forced:
        procs, cap = max(1, int(forced)), f"SNG_CPU_BASELINE_PROCS={forced}"
    elif quota is not None:
        procs, cap = min(affinity, quota), f"cgroup quota {quota} CPUs ({quota_src})"
    elif omp:
        procs, cap = max(1, min(affinity, int(omp))), f"no cgroup quota ({quota_src}); OMP_NUM_THREADS={omp}"
    else:
        procs, cap = affinity, f"no cgroup quota ({quota_src})"
    import oracle as O
    O.lib()   # build / load once in the parent: the forked workers inherit it
    with multiprocessing.get_context("fork").Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(kw, budget_s, w) for w in range(procs)])
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    per = [r[0] / r[1] for r in res]
    T = O.OracleConfig(**kw).T
    return {"value": steps / wall, "unit": "env-steps/s", "cores": procs, "kind": "port", "label": "restatement",
            "per_process": float(np.mean(per)),
            "sample": f"{steps // T} envs x 1 day (reset + {T} steps each), b-pv N={kw['number_of_chargers']} sparse "
                      f"{kw.get('time_interval', '1h')}; C restatement of the reference (oracle/), {procs} processes "
                      f"(sched_getaffinity {affinity} CPUs; {cap}), {wall:.1f} s",
            "cores_source": cap,
            "reference_python": {"value": [4700, 8200], "unit": "env-steps/s per core",
                                 "source": "SURVEY.md section 6: the reference's own step()+reset(), N=10, JSON I/O "
                                           "stubbed, in the build container (the reference does not exist on the "
                                           "GPU box)"}}


def rocprof_average_us(kernel, n_envs, chargers, build_id):
    """Average duration (us) of `kernel` in a committed rocprofv3 --stats summary taken on this very build
    (profiles/kernel_stats_index.json lists each summary with the build id of the library it measured,
    tools/pmc_summary.py), with the file it came from; (None, None) when no summary of this build exists
    (a stale summary of another build is never quoted)."""
    try:
        index = json.load(open(os.path.join(ROOT, "profiles", "kernel_stats_index.json")))
    except (OSError, ValueError):
        return None, None
    for e in reversed(index):   # the newest summary of this build and workload
        if e.get("build_id") != build_id or e.get("envs") != n_envs or e.get("chargers") != chargers:
            continue
        with open(os.path.join(ROOT, e["file"])) as fp:
            for line in fp:
                if line.startswith(f'"{kernel}('):
                    cols = line.rsplit('",', 1)[1].split(",")
                    return float(cols[2]) / 1e3, e["file"]
    return None, None


def load_pmc_traffic(n_envs, chargers, kernel, build_id):
    """Per-launch HBM bytes of the step kernel from the committed rocprofv3 PMC summary, only when it was
    collected on this build (its build id), for this kernel instantiation and size; else None."""
    path = os.path.join(ROOT, "profiles", "pmc_step_kernel.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    for e in reversed(d if isinstance(d, list) else [d]):
        if (e.get("envs") == n_envs and e.get("chargers") == chargers and e.get("kernel") == kernel
                and e.get("build_id") == build_id):
            return e.get("bytes_per_launch"), e.get("source")
    return None, None


def copy_ceiling(device, read_bytes, write_bytes, reps=50):
    """The measured bandwidth ceiling SURVEY.md 8(d) asks to quote beside the 8 TB/s spec: libsng's float4
    copy probe (sng_bandwidth_probe: one float4 per thread, nontemporal stores like the step) moving
    read_bytes + write_bytes per dispatch.  Returns GB/s for the dispatch's own device time (start/stop
    events per dispatch) and for back-to-back dispatches (start to start, as the day graphs run the step)."""
    import ctypes
    from smart_nanogrid_gym._native import check, lib
    d_us, b_us = ctypes.c_float(), ctypes.c_float()
    check(lib().sng_bandwidth_probe(device.index or 0, int(read_bytes), int(write_bytes), int(reps),
                                    ctypes.byref(d_us), ctypes.byref(b_us),
                                    ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)))
    tot = read_bytes + write_bytes
    return {"read_bytes": int(read_bytes), "write_bytes": int(write_bytes), "dispatch_us": round(d_us.value, 3),
            "back_to_back_us": round(b_us.value, 3), "gbs_dispatch": round(tot / (d_us.value * 1e-6) / 1e9, 1),
            "gbs_back_to_back": round(tot / (b_us.value * 1e-6) / 1e9, 1)}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, kw):
    """`bench.py --gpus N` (N > 1) without a launcher: measure the CPU baseline here, before anything
    touches the GPU, then start N fresh rank processes with torch.distributed.run (a child process, never
    an exec of this one) and return its exit code.  Rank 0 prints the JSON line with this process's
    cpu_baseline (handed over in a file named by SNG_BENCH_CPU_BASELINE)."""
    import subprocess
    import tempfile
    # the visible GPUs are counted in a child process, so this one never starts the HIP runtime
    # before its CPU baseline forks (whether torch.cuda.device_count() does is an implementation detail)
    probe = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True)
    ndev = int(probe.stdout.strip() or 0) if probe.returncode == 0 else 0
    if args.dist_backend == "nccl" and ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs for RCCL (one rank per GPU); "
              f"{ndev} visible (--dist-backend gloo shares them)", file=sys.stderr)
        return 2
    cpu = None if args.no_cpu_baseline else cpu_baseline(kw, args.cpu_budget)
    with tempfile.NamedTemporaryFile("w", suffix=".json", prefix="sng_cpu_baseline_", delete=False) as fp:
        json.dump(cpu, fp)
        cpu_file = fp.name
    env = dict(os.environ, SNG_BENCH_CPU_BASELINE=cpu_file, SNG_BENCH_LAUNCHER="bench.py --gpus (torch.distributed.run child)")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    try:
        return subprocess.run(cmd, env=env).returncode
    finally:
        os.unlink(cpu_file)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100, help="timed simulated days")
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--chargers", type=int, default=10)
    ap.add_argument("--time-interval", default="1h", help="'15min' with --extended-day = BASELINE config 5")
    ap.add_argument("--extended-day", action="store_true", help="build-defined days longer than 24 steps")
    ap.add_argument("--pv-noise", type=float, default=0.0, help="stochastic PV profile sigma (config 5: 0.2)")
    ap.add_argument("--price-noise", type=float, default=0.0, help="stochastic price profile sigma (config 5: 0.1)")
    ap.add_argument("--lanes", type=int, default=0, help="step kernel lanes per env (0 = library default)")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timing-days", type=int, default=3, help="eager days for the per-kernel HIP-event probe")
    ap.add_argument("--graph-days", type=int, default=20, help="days per graph replay (divides steps)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: RCCL over xGMI (default), or gloo with the day returns staged through host "
                         "memory (several ranks on one GPU, tests)")
    ap.add_argument("--v2x", action="store_true",
                    help="a V2X station (vehicle_to_everything): Box actions in [-1, 1], so most envs hit the "
                         "reference's V2X breakpoint every step (not the headline workload)")
    ap.add_argument("--per-env-flags", action="store_true",
                    help="time the step with the per-env per-step error-flag store of the diagnostics (the default "
                         "SngInfo watches the flag summary word instead)")
    args = ap.parse_args()

    E, N = args.envs, args.chargers
    kw = dict(number_of_chargers=N, time_interval=args.time_interval, charging_mode="bounded",
              vehicle_uncharged_penalty_mode="sparse", pv_system_available_in_model=True,
              battery_system_available_in_model=True)
    noise = args.pv_noise > 0 or args.price_noise > 0
    if args.v2x:
        kw.update(vehicle_to_everything=True)
    if args.extended_day or noise:
        kw.update(extended_day=args.extended_day, pv_noise=args.pv_noise, price_noise=args.price_noise)
    if args.gpus < 1:
        print(f"bench.py: --gpus must be >= 1 (got {args.gpus})", file=sys.stderr)
        return 2
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args, kw)   # N fresh rank processes; this one never touches the GPU
    world = int(env_world or "1")
    if world != args.gpus:   # an external launcher's world must be the one the line will report
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the CPU baseline is rank 0's report, measured before the GPU is initialised (forked workers, host
    # cores otherwise idle); under bench.py's own launcher the parent measured it before starting the ranks
    cpu, launcher = None, os.environ.get("SNG_BENCH_LAUNCHER", "external" if env_world else "none (N = 1)")
    if rank == 0 and not args.no_cpu_baseline:
        if os.environ.get("SNG_BENCH_CPU_BASELINE"):
            with open(os.environ["SNG_BENCH_CPU_BASELINE"]) as fp:
                cpu = json.load(fp)
        else:
            cpu = cpu_baseline(kw, args.cpu_budget)
    dist = None
    # one GPU per rank; ranks beyond the visible GPUs share them (gloo only: RCCL needs one rank per GPU).
    # torch.cuda.device_count() does not initialise the GPU on this image.
    ndev = max(1, torch.cuda.device_count())
    if world > 1 and args.dist_backend == "nccl" and ndev < world:
        print(f"bench.py: {world} RCCL ranks need {world} visible GPUs; {ndev} visible", file=sys.stderr)
        return 2
    gpu = local % ndev
    dist_info = {"backend": None, "world_size": 1, "launcher": launcher}
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "launcher": launcher}
        assert dist_info["world_size"] == args.gpus
    device = torch.device("cuda", gpu)
    torch.cuda.set_device(device)
    coll_dev = device if args.dist_backend == "nccl" else None   # where the collectives' tensors live

    from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv
    from smart_nanogrid_gym.parallel import DayReturnExchange, max_over_ranks, shard_envs

    offset, _ = shard_envs(world * E, world, rank)   # weak scaling: E envs per GPU, global ids
    venv = SmartNanogridVecEnv(E, seed=args.seed, device=gpu, rng="device", env_offset=offset,
                               step_lanes_per_env=args.lanes, **kw)
    T, A = venv.timesteps, venv.act_dim
    g = torch.Generator(device=device).manual_seed(args.seed + rank)
    low = torch.tensor(venv.action_space.low, device=device)
    high = torch.tensor(venv.action_space.high, device=device)
    acts = low + (high - low) * torch.rand((T, E, A), generator=g, device=device)
    acts = torch.where(torch.rand(acts.shape, generator=g, device=device) < 0.2, torch.zeros_like(acts), acts)
    acts = acts.contiguous()
    # the default SngInfo: the per-env error flags and the day return (for the all-gather), no diagnostics
    if args.per_env_flags:
        venv._info.flags = venv.flags_d.data_ptr()
    venv.reset_tensors(rng="device")
    kernel = venv.step_kernel_name()   # the instantiation the graphs below launch (device-RNG days)
    # days per graph replay (the same at every N, so per-GPU work is identical)
    D = max(1, args.graph_days)
    while args.steps % D:
        D -= 1
    xch = None
    if dist is not None:
        # N > 1: every day's per-env returns land in a [D, E] snapshot (one per graph, two
        # alternating graphs) and one RCCL all-gather per replay runs on the collective stream
        # while the next replay computes
        xch = DayReturnExchange(D, E, device, staging="device" if args.dist_backend == "nccl" else "host")
        graphs = [EpisodeGraph(venv, acts, with_reset=True, days=D, day_returns=xch.snap[k]) for k in range(2)]
    else:
        graphs = [EpisodeGraph(venv, acts, with_reset=True, days=D)]
    rep = [0]
    host_launch_s = []   # host time of each replay's hipGraphLaunch (the host must keep ahead of the device)

    def day():   # one graph replay = D simulated days
        k = rep[0] % len(graphs)
        if xch is not None:
            xch.acquire(k)
        h0 = time.perf_counter()
        graphs[k].launch()
        host_launch_s.append(time.perf_counter() - h0)
        if xch is not None:
            xch.gather(k)
        rep[0] += 1

    for _ in range(-(-args.warmup // D)):   # at least W warmup days
        day()
    host_launch_s.clear()
    if xch is not None:
        xch.finish()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()   # on the stream the graphs are launched on (torch's current stream)
    for _ in range(args.steps // D):
        day()
    if xch is not None:
        xch.finish()   # the last replay's gather is part of the timed work
    ev1.record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the step kernel's average duration as the graphs run it: the day's device time (HIP events
    # around the timed replays, on the graphs' stream) less the reset kernel, over the T step dispatches.
    # Inside a graph every dispatch starts when the previous one ends, so this is the start-to-start
    # time rocprofv3 --kernel-trace reports for the graph's step kernels.  The reset's own time and the
    # isolated per-dispatch step time come from HIP start/stop events attached to each dispatch
    # (hipExtLaunchKernel) over eager days of the same env/actions, right after the timed region.
    day_gpu_us = ev0.elapsed_time(ev1) * 1e3 / args.steps
    kernel_ms, reset_ms = venv.time_step_kernels(acts, days=args.timing_days, with_resets=True)
    reset_us = float(np.mean(reset_ms)) * 1e3
    graph_step_us = (day_gpu_us - reset_us) / T
    timing_src = (f"in-graph: (HIP-event device time per timed day {day_gpu_us:.2f} us - reset kernel "
                  f"{reset_us:.2f} us) / {T} step dispatches; reset and eager_launch_us from HIP start/stop "
                  f"events on each dispatch (hipExtLaunchKernel), {args.timing_days} eager days after the "
                  f"timed region, same stream/env/actions")
    elapsed = max_over_ranks(elapsed, device=coll_dev)
    # sanity: a day's returns are finite and <= 0
    ret = venv.return_d.cpu().numpy()
    assert np.isfinite(ret).all() and (ret <= 0).all()
    if xch is not None:   # every rank's returns of every day of the last replays arrived
        for k in range(2):
            got = xch.gathered(k).cpu().numpy()
            assert got.shape == (D, world * E) and np.isfinite(got).all() and (got <= 0).all() and (got < 0).any()

    if rank == 0:
        env_steps = world * E * T * args.steps
        value = env_steps / elapsed
        launch_s = graph_step_us * 1e-6
        eager_s = float(np.mean(kernel_ms)) * 1e-3
        bpl = survey_bytes(N) * E
        achieved = bpl / launch_s / 1e9
        rd, wr = step_kernel_bytes(N, noise, flags=args.per_env_flags)
        lpl = (rd + wr) * E
        from smart_nanogrid_gym._native import lib
        build_id = lib().sng_build_id().decode()
        traffic, traffic_src = load_pmc_traffic(E, N, kernel, build_id)
        rp_us, rp_file = rocprof_average_us(kernel, E, N, build_id)
        # measured ceilings: the same copy kernel at this step's own read/write bytes (one dispatch) and at
        # 1 GiB (512 MiB each way)
        c_step = copy_ceiling(device, rd * E, wr * E)
        c_big = copy_ceiling(device, 1 << 29, 1 << 29, reps=10)
        frac = lambda b, sec: round(b / sec / 1e9 / HBM_PEAK_GBS, 4)   # noqa: E731
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": kernel, "bytes_model": f"SURVEY.md 8(d) B(N) = 40N+65 = {survey_bytes(N)} B per env-step",
                "bytes_per_launch": bpl,
                "layout_bytes_model": f"this layout: {rd} B read + {wr} B written per env-step "
                                      f"(bench.step_kernel_bytes; per-env flag store {'on' if args.per_env_flags else 'off'})",
                "layout_bytes_per_launch": lpl,
                "frac_layout": frac(lpl, launch_s),
                "frac_pmc": None if traffic is None else frac(traffic, launch_s),
                "build_id": build_id,
                "traffic_source": (f"profiles/pmc_step_kernel.json, entry of build {build_id}: {traffic_src}; "
                                   "rocprofv3 FETCH_SIZE x2 gfx950 correction + WRITE_SIZE" if traffic is not None else
                                   f"no PMC passes committed for build {build_id} (profiles/pmc_step_kernel.json)"),
                "mean_launch_us": round(launch_s * 1e6, 3), "timing": timing_src,
                # the host side of the timed replays: a wall time per day well above the device time per day
                # means the host did not keep the GPU fed (one round-5 box: 0.25 against 0.17 ms)
                "host_launch_ms_per_replay": round(float(np.median(host_launch_s)) * 1e3, 4),
                "device_ms_per_day": round(day_gpu_us * 1e-3, 5),
                "eager_launch_us": round(eager_s * 1e6, 3), "reset_us": round(reset_us, 3),
                "frac_eager": frac(bpl, eager_s), "frac_layout_eager": frac(lpl, eager_s),
                "copy_step_size": c_step, "copy_1gib": c_big,
                "frac_of_copy_step_size": round(lpl / launch_s / 1e9 / c_step["gbs_back_to_back"], 4),
                "frac_of_copy_step_size_eager": round(lpl / eager_s / 1e9 / c_step["gbs_dispatch"], 4),
                "rocprof_avg_us": rp_us, "rocprof_file": rp_file,
                "frac_rocprof": None if rp_us is None else frac(bpl, rp_us * 1e-6),
                "frac_layout_rocprof": None if rp_us is None else frac(lpl, rp_us * 1e-6)}
        headline = (N == 10 and T == 24 and not noise and not args.v2x)
        metric = METRIC if headline else f"env-steps/sec (whole node) at N={E:,} envs × {N} chargers, {T}-step day"
        desc = ("v2x-" if args.v2x else "") + f"b-pv bounded sparse {args.time_interval}" + (
            (", extended day" if args.extended_day else "") +
            (f", stochastic PV/price profiles (sigma {args.pv_noise}/{args.price_noise})" if noise else ""))
        out = {"metric": metric, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
               "config": {"workload": f"{E} envs/GPU x {N} chargers x {T}-step day, {desc}, "
                                      f"GPU-RNG reset + {T} fused steps per bench step (hipGraph)",
                          "envs_per_gpu": E, "chargers": N, "timesteps": T,
                          "step_unit": "one simulated day of every env",
                          "days_per_graph_replay": D,
                          "parallelism": f"env-sharded x{world}" + (
                              (", RCCL all-gather of every day's returns, one per replay, overlapped"
                               if args.dist_backend == "nccl" else
                               ", gloo all-gather of every day's returns staged through host memory, one per replay")
                              if world > 1 else "")},
               "dist": dist_info, "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(out))
    for gr in graphs:
        gr.close()
    venv.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
