"""The N>1 path on CPU: world_size-2 gloo, env sharding by global index and the per-day
all-gather of returns.  The per-rank env simulation is the oracle here (the GPU envs are
covered by the gpu-marked sharding test); what this checks is the sharding arithmetic and
the collective: the gathered returns equal one process simulating the whole population."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from smart_nanogrid_gym.parallel import all_gather_returns, day_summary, max_over_ranks, shard_envs

KW = dict(number_of_chargers=4, time_interval="1h", charging_mode="bounded", vehicle_uncharged_penalty_mode="sparse")
TOTAL, SEED = 48, 321


def day_returns(global_ids):
    cfg = O.OracleConfig(**KW)
    out = []
    for g in global_ids:
        env = O.OracleEnv(cfg, SEED + int(g))
        env.reset()
        rng = np.random.default_rng(int(g))
        total = 0.0
        for t in range(cfg.T):
            a = rng.uniform(0, 1, cfg.act_dim).astype(np.float32)
            a[-1] = a[-1] * 2 - 1
            total += env.step(a)[1]
        out.append(total)
    return np.array(out)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = shard_envs(TOTAL, world, rank)
    local = torch.from_numpy(day_returns(range(off, off + cnt)))
    gathered = all_gather_returns(local)
    slowest = max_over_ranks(float(rank + 1))
    if rank == 0:
        q.put((gathered.numpy(), slowest, day_summary(gathered)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_envs_covers_population():
    for total, world in [(10, 3), (65536 * 8, 8), (7, 7), (100, 1)]:
        ranges = [shard_envs(total, world, r) for r in range(world)]
        assert ranges[0][0] == 0
        for (o1, c1), (o2, _) in zip(ranges, ranges[1:]):
            assert o1 + c1 == o2
        assert sum(c for _, c in ranges) == total
    with pytest.raises(ValueError):
        shard_envs(2, 4, 0)


def test_gloo_world2_gather_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, slowest, summary = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(gathered, day_returns(range(TOTAL)))
    assert slowest == 2.0
    assert summary["envs"] == TOTAL and summary["max_return"] <= 0


def _xch_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from smart_nanogrid_gym.parallel import DayReturnExchange
    days, envs = 3, 5
    x = DayReturnExchange(days, envs, torch.device("cpu"))
    results = []
    for rep in range(4):   # alternate buffers; each replay fills days x envs with rank/rep-tagged values
        k = rep % 2
        buf = x.acquire(k)
        buf.copy_(torch.arange(days * envs, dtype=torch.float64).reshape(days, envs) + 1000 * rank + 100 * rep)
        x.gather(k)
        if rep >= 1:   # the previous replay's gather, read after its buffer is reacquired
            x.acquire(1 - k)
            results.append(x.gathered(1 - k).clone())
    x.finish()
    results.append(x.gathered(1).clone())
    if rank == 0:
        q.put([r.numpy() for r in results])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_overlapped_day_return_exchange(world):
    """DayReturnExchange: double-buffered asynchronous all-gather of [days, E] day returns, at the world sizes the
    driver's scaling run uses (8 ranks as bench.py's 8 GPUs; gloo on the CPU here)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xch_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(results) == 4
    base = np.arange(15, dtype=np.float64).reshape(3, 5)
    for rep, got in enumerate(results):
        want = np.concatenate([base + 1000 * r + 100 * rep for r in range(world)], axis=1)
        np.testing.assert_array_equal(got, want)


def _unequal_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = shard_envs(5, world, rank)   # 3 and 2 envs: the single-buffer gather cannot take them
    try:
        all_gather_returns(torch.zeros(cnt, dtype=torch.float64))
        q.put((rank, "gathered"))
    except ValueError as e:
        q.put((rank, "ValueError" if "differ in size" in str(e) else str(e)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_unequal_shards_raise_on_every_rank():
    """unequal shards must fail on every rank together, before any mismatched collective."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_unequal_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == [(0, "ValueError"), (1, "ValueError")]
