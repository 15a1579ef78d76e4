"""Multi-GPU sharding of one env population (one process per GPU, torch.distributed).

Envs are independent, so the population is split into contiguous global index ranges, one
per rank; each rank's SmartNanogridVecEnv gets env_offset = the start of its range, which
makes every env's random streams depend on its global index only (a sharded run reproduces
the single-GPU run).  There is no per-step communication: once per simulated day the ranks
exchange the per-env day returns with one all-gather (RCCL over xGMI with the "nccl"
backend; gloo on CPU for tests).
"""
import torch
import torch.distributed as dist


def shard_envs(total_envs, world_size, rank):
    """Contiguous [offset, offset + count) range of global env ids owned by `rank`."""
    if total_envs < world_size:
        raise ValueError("fewer envs than ranks")
    base, extra = divmod(int(total_envs), int(world_size))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def all_gather_returns(local, group=None):
    """Gather every rank's per-env returns into one [total_envs] tensor in global env order.
    Shards must be equal-sized (weak scaling) for the single-buffer collective."""
    world = dist.get_world_size(group)
    out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    try:
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    except (RuntimeError, NotImplementedError, AttributeError):   # backends without the fused form
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local.contiguous(), group=group)
        out = torch.cat(parts)
    return out


class DayReturnExchange:
    """The all-gather of one graph replay's day returns ([days, E] per rank -> [world, days, E]),
    issued asynchronously so it runs on the collective stream while the next replay's kernels
    run.  Two snapshot buffers alternate (one EpisodeGraph per buffer, via its day_returns):
    before buffer k is refilled, acquire(k) makes the compute stream wait for the gather that
    reads it (work.wait() orders streams; the host does not block on NCCL/RCCL)."""

    def __init__(self, days, envs, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.snap = [torch.zeros((days, envs), dtype=torch.float64, device=device) for _ in range(2)]
        self.out = [torch.empty((self.world, days, envs), dtype=torch.float64, device=device) for _ in range(2)]
        self.work = [None, None]
        self.gathers = 0

    def acquire(self, k):
        """Snapshot buffer k for the next replay, once its previous gather has read it."""
        if self.work[k] is not None:
            self.work[k].wait()
            self.work[k] = None
        return self.snap[k]

    def gather(self, k):
        """Start the all-gather of buffer k (after the replay that fills it has been launched)."""
        try:
            self.work[k] = dist.all_gather_into_tensor(self.out[k], self.snap[k], group=self.group, async_op=True)
        except (RuntimeError, NotImplementedError, AttributeError):   # backends without the fused form
            self.work[k] = dist.all_gather(list(self.out[k].unbind(0)), self.snap[k], group=self.group,
                                           async_op=True)
        self.gathers += 1

    def finish(self):
        for k in range(2):
            if self.work[k] is not None:
                self.work[k].wait()
                self.work[k] = None

    def gathered(self, k):
        """[days, world * E]: every rank's returns in global env order, per day."""
        w, d, e = self.out[k].shape
        return self.out[k].permute(1, 0, 2).reshape(d, w * e)


def max_over_ranks(value, device=None, group=None):
    """Max of a host float over ranks (bench timing: the slowest rank defines the wall time)."""
    if not dist.is_available() or not dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def day_summary(returns):
    """Population statistics of one day's returns (the quantity the reference's evaluator plots)."""
    r = returns.double()
    return {"envs": int(r.numel()), "mean_return": float(r.mean()), "min_return": float(r.min()),
            "max_return": float(r.max())}
