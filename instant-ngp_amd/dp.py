"""Data-parallel training over the GPUs of one node: one process per GPU,
torch.distributed with the "nccl" backend (= RCCL over xGMI on ROCm), one all-reduce of the
contiguous fp16 gradient buffer per step (widened to fp32 on the wire, rounded once), the 1/N average
folded into the optimizer's loss scale.

The reference trains on one GPU only (multi-GPU is render replication); this module is
the new exchange step. Sharding keeps the *global* ray index i so every rank draws exactly the rays
the 1-GPU run would draw (rng.advance(i * N_MAX_RANDOM_SAMPLES_PER_RAY), src/testbed_nerf.cu:1417-1421).
"""
import ctypes as C
import os
import sys
import traceback

import torch
import torch.distributed as dist

# ngp_allreduce_fn (include/ngp_engine.h): int (*)(void* user, void* buf, uint64_t count, int dtype, int op, void* stream)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_void_p)


def init_from_env(backend=None):
    """Initialise the process group from RANK/WORLD_SIZE/MASTER_* (torch.distributed.run)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {"device_id": torch.device("cuda", local_rank)} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return rank, world, local_rank


def shard_range(n_global, rank, world):
    """Contiguous shard [lo, hi) of n_global items for `rank`; shards partition [0, n_global)."""
    lo = n_global * rank // world
    hi = n_global * (rank + 1) // world
    return lo, hi


def allreduce_gradients(grads, world, group=None):
    """Sum the gradient buffer over ranks in place (RCCL all-reduce). Returns the loss-scale factor
    the optimizer must divide by (world) so that the update uses the mean gradient."""
    if world > 1:
        dist.all_reduce(grads, op=dist.ReduceOp.SUM, group=group)
    return float(world)


def allreduce_counters(values, world):
    """All-reduce the per-step scalars (measured sample counts, loss sum) used by the rays-per-batch
    adaptation (NerfCounters::update_after_training, src/testbed_nerf.cu:3583-3609)."""
    on_gpu = dist.is_initialized() and dist.get_backend() == "nccl"
    t = torch.as_tensor(values, dtype=torch.float64, device="cuda" if on_gpu else "cpu")
    if world > 1:
        dist.all_reduce(t)
    return t.cpu().tolist()


class _stdout_to_stderr:
    """Redirect file descriptor 1 to 2 (native libraries write there directly, below sys.stdout)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


class EngineComm:
    """The engine's own RCCL communicator (ngp_dp_comm_*): rank 0 makes the unique id, torch.distributed
    broadcasts it, every rank joins. `fn`/`user` plug into the engine's exchange hooks
    (ngp_trainer_set_allreduce, ngp_nerf_trainer_set_data_parallel), so the all-reduce is issued by the
    engine on its own stream — inside a captured HIP graph if the step is captured."""

    def __init__(self, rank, world, group=None, wire="f32"):
        from ._capi import check, lib
        with _stdout_to_stderr():  # RCCL prints its version banner to stdout: keep bench.py's one JSON line clean
            self._init(rank, world, group, wire, check, lib)

    def _init(self, rank, world, group, wire, check, lib):
        idb = (C.c_uint8 * 128)()
        if rank == 0:
            check(lib().ngp_dp_comm_unique_id(idb))
        if world > 1 or dist.is_initialized():
            t = torch.tensor(list(idb), dtype=torch.uint8)
            if dist.get_backend(group) == "nccl":
                t = t.cuda()
            dist.broadcast(t, src=0, group=group)
            idb = (C.c_uint8 * 128)(*t.cpu().tolist())  # else a world of one: no process group needed
        h = C.c_void_p()
        check(lib().ngp_dp_comm_create(rank, world, idb, C.byref(h)))
        self.handle, self.rank, self.world = h, rank, world
        # fp16 gradient sums travel widened to fp32 and are rounded once (ngp_dp_comm_set_wire)
        check(lib().ngp_dp_comm_set_wire(h, {"f32": 0, "f16": 1}[wire]))
        self.wire = wire
        self.fn = C.cast(lib().ngp_dp_comm_allreduce, C.c_void_p)

    def allreduce(self, tensor, op="sum", stream=None):
        from ._capi import check, lib
        dt = {torch.float32: 0, torch.float16: 1}[tensor.dtype]
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        check(lib().ngp_dp_comm_allreduce(self.handle, C.c_void_p(tensor.data_ptr()), tensor.numel(), dt,
                                          0 if op == "sum" else 1, C.c_void_p(s)))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                from ._capi import lib
                lib().ngp_dp_comm_destroy(h)
            except Exception:
                pass
            self.handle = None


def _host_allreduce(t, op, group, stream):
    """All-reduce a device tensor through torch.distributed on the host: wait for `stream`, sum (or max)
    a float32 host copy, write it back and wait for the copy (gloo: CPU tests, ranks sharing a GPU)."""
    (torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()).synchronize()
    h = t.float().cpu()
    dist.all_reduce(h, op=op, group=group)
    t.copy_(h.to(t.dtype))
    torch.cuda.synchronize()


REDUCE_SCATTER_SUM, ALL_GATHER = 2, 3  # ngp_engine.h: the sharded optimizer's hook ops


def _host_shard_collective(t, op, group, stream):
    """NGP_REDUCE_SCATTER_SUM / NGP_ALL_GATHER on a device tensor, in place (rank r's slice is the r-th of world
    equal slices). nccl: torch.distributed's collectives on `stream`; gloo: host round trip (the reduce-scatter as
    a float32 all-reduce of the whole buffer, which leaves every slice summed; the all-gather bit-exact)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    c = t.numel() // world
    if dist.get_backend(group) == "nccl":
        s = torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()
        with torch.cuda.stream(s):
            if op == REDUCE_SCATTER_SUM:
                out = torch.empty(c, dtype=t.dtype, device=t.device)
                dist.reduce_scatter_tensor(out, t, group=group)
                t[rank * c:(rank + 1) * c].copy_(out)
            else:
                dist.all_gather_into_tensor(t, t[rank * c:(rank + 1) * c].clone(), group=group)
        return
    (torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()).synchronize()
    if op == REDUCE_SCATTER_SUM:
        h = t.float().cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h.to(t.dtype))
    else:
        # gloo gathers float32 (not 16-bit types): fp16 slices travel widened, which is exact both ways
        parts = [torch.empty(c, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(parts, t[rank * c:(rank + 1) * c].float().cpu().contiguous(), group=group)
        t.copy_(torch.cat(parts).to(t.device, t.dtype))
    torch.cuda.synchronize()


def make_allreduce_callback(group=None, timer=None):
    """The engine's exchange hook (ngp_nerf_trainer_set_data_parallel) over torch.distributed.

    nccl (= RCCL over xGMI): the all-reduce is enqueued on the engine's stream. gloo (CPU tests, or
    several ranks sharing one GPU): host round trip, summed in fp32. `timer` (optional) gets
    `add(ms)` per host round trip. Keep the returned object alive while the engine may call it."""
    from .network import wrap_device
    import time

    def cb(user, ptr, count, dtype, op, stream):
        try:
            t = wrap_device(ptr, int(count), torch.float32 if dtype == 0 else torch.float16)
            if op in (REDUCE_SCATTER_SUM, ALL_GATHER):  # the sharded optimizer's collectives (in place)
                t0 = time.perf_counter()
                _host_shard_collective(t, op, group, stream)
                if timer is not None:
                    timer.add(1e3 * (time.perf_counter() - t0))
                return 0
            rop = dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX
            if dist.get_backend(group) == "nccl":
                s = torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()
                with torch.cuda.stream(s):
                    dist.all_reduce(t, op=rop, group=group)
            else:
                t0 = time.perf_counter()
                _host_allreduce(t, rop, group, stream)
                if timer is not None:
                    timer.add(1e3 * (time.perf_counter() - t0))
            return 0
        except Exception:
            traceback.print_exc(file=sys.stderr)
            return -1

    return ALLREDUCE_FN(cb)


class HostComm:
    """Gradient exchange through torch.distributed with a host round trip (gloo backend): the same
    interface as EngineComm (`world`, `fn`/`handle` for the engine's exchange hooks, `allreduce(tensor)`)
    for ranks that share one GPU or run without RCCL. Not capturable into a HIP graph (the hook
    synchronises the stream). Times its own round trips (`ms`, `calls`): the engine profiler sees only
    device work."""

    def __init__(self, rank, world, group=None):
        self.rank, self.world, self.group = rank, world, group
        self.ms, self.calls = 0.0, 0
        self._cb = make_allreduce_callback(group, timer=self)
        self.fn = C.cast(self._cb, C.c_void_p)
        self.handle = None
        self.wire = "f32"

    def add(self, ms):
        self.ms += ms
        self.calls += 1

    def reset_timer(self):
        self.ms, self.calls = 0.0, 0

    def allreduce(self, tensor, op="sum", stream=None):
        import time
        t0 = time.perf_counter()
        _host_allreduce(tensor, dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX, self.group,
                        stream if stream is not None else torch.cuda.current_stream().cuda_stream)
        self.add(1e3 * (time.perf_counter() - t0))


def make_comm(rank, world, group=None, wire="f32"):
    """The gradient exchange for this process group: the engine's RCCL communicator under the nccl
    backend, a host round trip (HostComm) under gloo."""
    if dist.get_backend(group) == "nccl":
        return EngineComm(rank, world, group, wire=wire)
    return HostComm(rank, world, group)


def reduce_scalar(value, op="max", group=None):
    """All-reduce one float over the ranks (a device tensor under nccl, a host tensor under gloo)."""
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN}[op], group=group)
    return float(t.item())
