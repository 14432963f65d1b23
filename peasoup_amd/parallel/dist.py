"""Process-group plumbing for one-process-per-GPU runs.

The reference is a single process with one pthread per GPU and no
collectives (src/pipeline_multi.cu:33-259: DMDispenser mutex queue, host-side
concatenation of per-worker candidate vectors after pthread_join).  Here each
GPU is its own rank; ``torch.distributed`` with the ``nccl`` backend is RCCL
over xGMI on ROCm.  Collectives used by the pipeline:

* filterbank broadcast (packed bytes, rank 0 -> all)          ``broadcast_bytes``
* per-rank candidate gather (serialised candidate trees)      ``gather_bytes``
* multi-beam coincidence counts (uint8 indicator sums)        ``all_reduce_sum``
* fold-job results (per-candidate fold records)               ``gather_bytes``

On a CPU box (tests) the same code runs on the ``gloo`` backend.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    forced: bool = False  # PSOUP_FORCE_PG: a process group (and every collective) at world size 1

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return (self.world_size > 1 or self.forced) and dist.is_available() and dist.is_initialized()


_CTX: Optional[DistContext] = None


def init(backend: Optional[str] = None, timeout_s: float = 1800.0) -> DistContext:
    """Initialise (or return) the process group from torchrun-style env vars.

    ``backend`` defaults to ``nccl`` (RCCL) when a GPU is visible, else
    ``gloo``.  A single process (WORLD_SIZE unset or 1) needs no rendezvous,
    unless ``PSOUP_FORCE_PG=1``: then a world-1 process group is created and
    every collective of the pipeline (filterbank broadcast, candidate gather,
    reductions, barriers) really runs through RCCL on the one GPU.
    """
    global _CTX
    if _CTX is not None:
        return _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    has_gpu = torch.cuda.is_available() and torch.cuda.device_count() > 0
    if backend is None:
        # PSOUP_DIST_BACKEND=gloo rehearses multi-rank runs with several ranks on one GPU
        backend = os.environ.get("PSOUP_DIST_BACKEND") or ("nccl" if has_gpu else "gloo")
    device = torch.device("cpu")
    if has_gpu and backend == "nccl":
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local % ndev)
        device = torch.device("cuda", local % ndev)
    elif has_gpu:
        device = torch.device("cuda", local % torch.cuda.device_count())
        torch.cuda.set_device(device)
    forced = world == 1 and os.environ.get("PSOUP_FORCE_PG", "0") not in ("", "0")
    if (world > 1 or forced) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        kwargs = dict(backend=backend, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = device
        dist.init_process_group(**kwargs)
    _CTX = DistContext(rank=rank, world_size=world, local_rank=local,
                       backend=backend if (world > 1 or forced) else "none", device=device, forced=forced)
    try:
        from .. import _C

        _C.set_log_rank(rank if world > 1 else -1)
    except Exception:  # pragma: no cover
        pass
    return _CTX


def context() -> DistContext:
    return _CTX if _CTX is not None else init()


def shutdown() -> None:
    global _CTX
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _CTX = None


def barrier() -> None:
    ctx = context()
    if ctx.distributed:
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


def _comm_device(ctx: DistContext) -> torch.device:
    return ctx.device if ctx.backend == "nccl" else torch.device("cpu")


def broadcast_bytes(buf: Optional[torch.Tensor], nbytes: int, src: int = 0) -> torch.Tensor:
    """Broadcast a uint8 buffer of ``nbytes`` from ``src`` (RCCL over xGMI on GPUs).

    Non-root ranks may pass ``None``; a destination buffer is allocated on the
    communication device.  Large buffers are sent in 1 GiB pieces.
    """
    ctx = context()
    dev = _comm_device(ctx)
    if buf is None:
        buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    if not ctx.distributed:
        return buf
    assert buf.dtype == torch.uint8 and buf.numel() >= nbytes
    piece = 1 << 30
    flat = buf.view(-1)
    for off in range(0, nbytes, piece):
        part = flat[off:min(nbytes, off + piece)]
        if part.is_cuda and ctx.backend != "nccl":  # gloo: stage through host memory
            h = part.cpu()
            dist.broadcast(h, src=src)
            part.copy_(h)
        else:
            dist.broadcast(part, src=src)
    return buf


def gather_bytes(payload: bytes, dst: Optional[int] = 0) -> Optional[List[bytes]]:
    """Variable-length gather of byte strings (all_gather of sizes, then of a
    padded uint8 tensor).  Returns the list on ``dst`` (all ranks if dst is
    None), else None."""
    ctx = context()
    if not ctx.distributed:
        return [payload]
    dev = _comm_device(ctx)
    n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(ctx.world_size)]
    dist.all_gather(sizes, n)
    sizes_i = [int(s.item()) for s in sizes]
    mx = max(1, max(sizes_i))
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    if payload:
        buf[: len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    outs = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(ctx.world_size)]
    dist.all_gather(outs, buf)
    if dst is not None and ctx.rank != dst:
        return None
    return [bytes(o[:s].cpu().numpy().tobytes()) for o, s in zip(outs, sizes_i)]


def broadcast_object_bytes(payload: Optional[bytes], src: int = 0) -> bytes:
    """Broadcast a byte string of unknown length from ``src``."""
    ctx = context()
    if not ctx.distributed:
        return payload or b""
    dev = _comm_device(ctx)
    n = torch.tensor([len(payload) if ctx.rank == src and payload else 0], dtype=torch.int64, device=dev)
    dist.broadcast(n, src=src)
    size = int(n.item())
    buf = torch.zeros(max(1, size), dtype=torch.uint8, device=dev)
    if ctx.rank == src and size:
        buf[:size] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    dist.broadcast(buf, src=src)
    return bytes(buf[:size].cpu().numpy().tobytes())


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    """In-place sum across ranks (RCCL ring/tree all-reduce over xGMI)."""
    ctx = context()
    if ctx.distributed:
        if ctx.backend != "nccl" and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h)
            t.copy_(h)
        else:
            dist.all_reduce(t)
    return t


def all_reduce_max_float(x: float) -> float:
    ctx = context()
    if not ctx.distributed:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_comm_device(ctx))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_range(n: int, world: int, rank: int, weights: Optional[Sequence[float]] = None) -> range:
    """Contiguous shard of ``range(n)`` for ``rank``; with ``weights`` the cut
    points balance the summed weight (e.g. acceleration trials per DM)."""
    if world <= 1:
        return range(n)
    if weights is None:
        base, rem = divmod(n, world)
        start = rank * base + min(rank, rem)
        return range(start, start + base + (1 if rank < rem else 0))
    w = [float(x) for x in weights]
    assert len(w) == n
    total = sum(w)
    cuts = [0]
    acc = 0.0
    k = 1
    for i, x in enumerate(w):
        acc += x
        while k < world and acc >= total * k / world:
            cuts.append(i + 1)
            k += 1
    while len(cuts) < world:
        cuts.append(n)
    cuts.append(n)
    return range(cuts[rank], cuts[rank + 1])


_QUEUE_SEQ: dict = {}


class WorkQueue:
    """First-come work queue shared by every rank: ``claim()`` hands out the
    indices ``0 .. n-1``, each to exactly one rank, then ``None``.

    The cross-process form of the reference's ``DMDispenser``
    (src/pipeline_multi.cu:33-81: a mutex-guarded "next DM" counter read by one
    pthread per GPU).  Here the counter is an atomic ``add`` on the
    process group's host-side key-value store (the c10d TCPStore torchrun set
    up), so claiming a DM chunk costs one small TCP round trip to rank 0's
    store and no GPU collective; fast ranks simply claim more chunks.

    Every rank must create its queues in the same order (the key is
    ``name`` plus a per-name sequence number, so a queue re-created by a later
    step starts from zero).  Without a process group the queue is a local
    counter.
    """

    def __init__(self, name: str, n: int):
        self.n = int(n)
        seq = _QUEUE_SEQ.get(name, 0)
        _QUEUE_SEQ[name] = seq + 1
        self.key = f"psoup/queue/{name}/{seq}"
        self._local = 0
        self._store = None
        ctx = context()
        if ctx.distributed:
            from torch.distributed import distributed_c10d

            self._store = distributed_c10d._get_default_store()
        self.claimed: List[int] = []

    def claim(self) -> Optional[int]:
        if self._store is not None:
            i = int(self._store.add(self.key, 1)) - 1
        else:
            i = self._local
            self._local += 1
        if i >= self.n:
            return None
        self.claimed.append(i)
        return i
