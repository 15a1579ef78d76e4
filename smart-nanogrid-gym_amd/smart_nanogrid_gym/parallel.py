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


def _fused_gather(group=None):
    """all_gather_into_tensor on RCCL/NCCL; the list form elsewhere (gloo).  Chosen from the backend, which
    every rank of the group shares, so all ranks issue the same collective."""
    return dist.get_backend(group) == "nccl"


def check_equal_shards(count, device=None, group=None):
    """The single-buffer gathers need the same number of envs on every rank (weak scaling); shard_envs
    gives unequal counts when total % world != 0.  One all-reduce of (count, -count) tells every rank the
    max and min, so every rank raises together instead of one rank entering a mismatched collective."""
    t = torch.tensor([float(count), -float(count)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    if t[0].item() != -t[1].item():
        raise ValueError(f"env shards differ in size across ranks ({int(-t[1].item())}..{int(t[0].item())}): "
                         "use a total divisible by the world size")


def all_gather_returns(local, group=None):
    """Gather every rank's per-env returns into one [total_envs] tensor in global env order.
    Shards must be equal-sized (weak scaling); checked on every rank first."""
    world = dist.get_world_size(group)
    local = local.contiguous()
    check_equal_shards(local.numel(), device=local.device, group=group)
    if _fused_gather(group):
        out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local, group=group)
        return out
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local, group=group)
    return torch.cat(parts)


class DayReturnExchange:
    """The all-gather of one graph replay's day returns ([days, E] per rank -> [world, days, E]),
    issued asynchronously so it runs on the collective stream while the next replay's kernels
    run.  Two snapshot buffers alternate (one EpisodeGraph per buffer, via its day_returns):
    before buffer k is refilled, acquire(k) makes the compute stream wait for the gather that
    reads it (work.wait() orders streams; the host does not block on NCCL/RCCL).

    staging="host" (gloo, which gathers host tensors; several ranks sharing one GPU): gather(k) copies
    the snapshot into pinned host memory once the replay that fills it is done and gathers that copy, so
    acquire(k) has nothing left to wait for on the device."""

    def __init__(self, days, envs, device, group=None, staging="device"):
        self.group = group
        self.world = dist.get_world_size(group)
        self.host = staging == "host"
        check_equal_shards(envs, device=None if self.host else device, group=group)
        self.fused = _fused_gather(group) and not self.host
        self.snap = [torch.zeros((days, envs), dtype=torch.float64, device=device) for _ in range(2)]
        odev = "cpu" if self.host else device
        self.out = [torch.empty((self.world, days, envs), dtype=torch.float64, device=odev) for _ in range(2)]
        self.staged = ([torch.empty((days, envs), dtype=torch.float64, pin_memory=True) for _ in range(2)]
                       if self.host else None)
        self.work = [None, None]
        self.gathers = 0

    def acquire(self, k):
        """Snapshot buffer k for the next replay, once its previous gather has read it."""
        if self.work[k] is not None:
            self.work[k].wait()
            self.work[k] = None
        return self.snap[k]

    def gather(self, k, stream=None):
        """Start the all-gather of buffer k (after the replay that fills it has been launched).  stream: the
        stream that replay was launched on (a torch.cuda.Stream or a raw hipStream_t handle, as given to
        EpisodeGraph.launch), when it is not the current stream: the current stream then waits for it, so
        the copy or collective below cannot read a half-filled snapshot."""
        on_gpu = self.snap[k].is_cuda
        cur = torch.cuda.current_stream(self.snap[k].device) if on_gpu else None
        if stream is not None and on_gpu:
            if not isinstance(stream, torch.cuda.Stream):
                stream = torch.cuda.ExternalStream(int(stream), device=self.snap[k].device)
            if stream != cur:
                ev = torch.cuda.Event()
                ev.record(stream)
                cur.wait_event(ev)
        if self.host:
            self.staged[k].copy_(self.snap[k], non_blocking=True)
            if on_gpu:
                cur.synchronize()
            self.work[k] = dist.all_gather(list(self.out[k].unbind(0)), self.staged[k], group=self.group,
                                           async_op=True)
        elif self.fused:
            self.work[k] = dist.all_gather_into_tensor(self.out[k], self.snap[k], group=self.group, async_op=True)
        else:
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


class NativeComm:
    """The C ABI's own RCCL exchange (sng_comm_create / sng_allgather_returns in include/sng.h) -- the
    multi-GPU path a non-Python host uses.  Here the unique id travels over an existing
    torch.distributed group (rank 0 makes it); a C host would use a file, a socket or MPI."""

    def __init__(self, device, group=None):
        import ctypes
        from ._native import COMM_ID_BYTES, lib
        self._lib = lib()
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        if rank == 0:
            self._check(self._lib.sng_comm_unique_id(buf), None)
        ids = [buf.raw if rank == 0 else None]
        dist.broadcast_object_list(ids, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        h = ctypes.c_void_p()
        self._check(self._lib.sng_comm_create(int(device), world, rank, ids[0], ctypes.byref(h)), None)
        self._h, self.world, self.rank, self.device = h, world, rank, int(device)

    def _check(self, rc, handle):
        if rc != 0:
            msg = self._lib.sng_comm_last_error(handle)
            raise RuntimeError(f"sng comm error {rc}: {msg.decode() if msg else ''}")

    def all_gather_returns(self, local, out=None):
        """[count] f64 device tensor per rank -> [world * count], rank-major, on the current stream."""
        import ctypes
        local = local.contiguous()
        if out is None:
            out = torch.empty(self.world * local.numel(), dtype=torch.float64, device=local.device)
        stream = ctypes.c_void_p(torch.cuda.current_stream(local.device).cuda_stream)
        self._check(self._lib.sng_allgather_returns(self._h, ctypes.c_void_p(local.data_ptr()),
                                                    ctypes.c_void_p(out.data_ptr()), local.numel(), stream), self._h)
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._lib.sng_comm_destroy(self._h)
            self._h = None


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
