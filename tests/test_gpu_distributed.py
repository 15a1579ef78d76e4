"""GPU + gloo: the multi-rank path with the real library.  Two ranks (processes) share the one GPU of
the box, each holding its shard of one env population (env_offset from parallel.shard_envs), replay two
device-RNG days as the bench does (EpisodeGraph with per-day return rows) and all-gather the day
returns over gloo.  The gathered returns must equal one handle simulating the whole population: the
sharding is exact, so the RCCL run of the 8-GPU bench gathers the same numbers."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

KW = dict(number_of_chargers=10, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
E_RANK, SEED, DAYS, WORLD = 4096, 31, 2, 2


def _actions(total, device):
    g = torch.Generator(device=device).manual_seed(5)
    a = torch.rand((24, total, 11), generator=g, device=device)
    a[..., -1] = a[..., -1] * 2 - 1
    return a


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv
        from smart_nanogrid_gym.parallel import all_gather_returns, shard_envs
        off, cnt = shard_envs(world * E_RANK, world, rank)
        dev = torch.device("cuda", 0)
        acts = _actions(world * E_RANK, dev)[:, off:off + cnt].contiguous()
        venv = SmartNanogridVecEnv(cnt, seed=SEED, rng="device", env_offset=off, **KW)
        rows = torch.zeros((DAYS, cnt), dtype=torch.float64, device=dev)
        g = EpisodeGraph(venv, acts, days=DAYS, day_returns=rows)
        g.launch()
        torch.cuda.synchronize()
        gathered = [all_gather_returns(rows[d].cpu()) for d in range(DAYS)]   # gloo: host tensors
        g.close()
        venv.close()
        if rank == 0:
            q.put(np.stack([x.numpy() for x in gathered]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_one_gpu_gather_equals_one_population():
    import torch.multiprocessing as mp
    from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    total = WORLD * E_RANK
    dev = torch.device("cuda", 0)
    full = SmartNanogridVecEnv(total, seed=SEED, rng="device", **KW)
    rows = torch.zeros((DAYS, total), dtype=torch.float64, device=dev)
    g = EpisodeGraph(full, _actions(total, dev), days=DAYS, day_returns=rows)
    g.launch()
    torch.cuda.synchronize()
    want = rows.cpu().numpy()
    g.close()
    full.close()
    assert gathered.shape == (DAYS, total)
    np.testing.assert_array_equal(gathered, want)
    assert np.isfinite(want).all() and (want < 0).mean() > 0.99


def test_native_rccl_exchange_world1():
    """The C ABI's own RCCL exchange (sng_comm_create / sng_allgather_returns), world 1 on this box: the
    gathered buffer is the rank's day returns (the 8-GPU gather is the driver's run)."""
    import torch.distributed as dist
    from smart_nanogrid_gym import EpisodeGraph, SmartNanogridVecEnv
    from smart_nanogrid_gym.parallel import NativeComm
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        comm = NativeComm(0)
        venv = SmartNanogridVecEnv(E_RANK, seed=SEED, rng="device", **KW)
        rows = torch.zeros((DAYS, E_RANK), dtype=torch.float64, device=dev)
        g = EpisodeGraph(venv, _actions(E_RANK, dev), days=DAYS, day_returns=rows)
        g.launch()
        out = comm.all_gather_returns(rows.reshape(-1))
        torch.cuda.synchronize()
        assert torch.equal(out, rows.reshape(-1)) and bool((out < 0).any())
        comm.close()
        g.close()
        venv.close()
    finally:
        dist.destroy_process_group()


def test_bench_world2_branch_on_one_gpu():
    """bench.py's own world > 1 branch (process group, two alternating day graphs writing
    per-day return rows, the overlapped DayReturnExchange, max-over-ranks timing and the gathered-returns
    asserts) run by torch.distributed.run with two ranks sharing this box's one GPU.  RCCL needs a GPU per
    rank, so the ranks gather over gloo with the snapshots staged through host memory
    (--dist-backend gloo); the 8-GPU driver run takes the RCCL path of the same code."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "2", "--envs", "4096", "--dist-backend", "gloo",
           "--no-cpu-baseline", "--timing-days", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 4 and out["value"] > 0
    assert out["config"]["envs_per_gpu"] == 4096 and "env-sharded x2" in out["config"]["parallelism"]
    assert out["dist"] == {"backend": "gloo", "world_size": 2, "launcher": "external"}


def test_bench_gpus2_launches_its_own_ranks():
    """`bench.py --gpus 2` with no launcher measures the CPU baseline itself (a short
    budget here), then starts two fresh rank processes (torch.distributed.run as a child) that share this
    box's GPU over gloo.  Rank 0's line reports n_gpus 2, the initialised world size and the parent's
    cpu_baseline."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "2",
           "--envs", "4096", "--dist-backend", "gloo", "--cpu-budget", "1", "--timing-days", "1"]
    env = dict(os.environ, SNG_CPU_BASELINE_PROCS="2")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and "env-sharded x2" in out["config"]["parallelism"]
    assert out["dist"]["world_size"] == 2 and out["dist"]["backend"] == "gloo"
    assert out["dist"]["launcher"].startswith("bench.py --gpus")
    assert out["cpu_baseline"]["cores"] == 2 and out["cpu_baseline"]["value"] > 0
