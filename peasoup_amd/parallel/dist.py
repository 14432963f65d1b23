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

Peer-failure handling (the reference throws and terminates,
include/utils/exceptions.hpp:13-153).  A multi-rank group must not leave its
surviving ranks blocked in a collective when one rank fails:

* ``report_failure(msg)``: a failing rank publishes "rank r: msg" under one
  key of the rendezvous store before it exits non-zero;
* a watchdog thread on every rank polls that key and the peers' heartbeat
  counters (``PSOUP_HEARTBEAT_S``, default 1 s); on a published failure, on a
  peer whose counter has not moved for ``PSOUP_PEER_TIMEOUT`` seconds
  (default 60: a peer killed without reporting), or when the store itself is
  gone (rank 0 died), it prints the cause with this rank's context and ends
  the process with exit code 3 -- which tears down its RCCL communicator (the
  ``ncclCommAbort`` equivalent) instead of waiting in a collective;
* every collective is also bounded by the process-group timeout
  (``PSOUP_COLLECTIVE_TIMEOUT``, default 1800 s) as the last backstop.
No re-exec and no in-process restart: recovery is a re-run (or torchrun's
``--max-restarts``) with ``--checkpoint_dir``, which resumes from the per-DM
spill files.
"""
from __future__ import annotations

import datetime
import os
import sys
import threading
import time
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


_ABORT_KEY = "psoup/abort"
_WATCHDOG: Optional["_Watchdog"] = None


class _Watchdog(threading.Thread):
    """Heartbeat + failure watch over the rendezvous store (see module doc)."""

    def __init__(self, store, rank: int, world: int, period: float, peer_timeout: float):
        super().__init__(name="psoup-watchdog", daemon=True)
        self.store, self.rank, self.world = store, rank, world
        self.period, self.peer_timeout = period, peer_timeout
        self.stop = threading.Event()
        self.beats = 0

    def _abort(self, why: str) -> None:
        sys.stderr.write(f"[rank {self.rank}] aborting: {why}\n")
        sys.stderr.flush()
        sys.stdout.flush()
        if self.rank == 0:
            # rank 0 hosts the store: keep it up a few polls so every peer
            # reads the failure record instead of a vanished store
            time.sleep(max(1.0, 5 * self.period))
        os._exit(3)

    def run(self) -> None:
        seen = {r: (-1, time.monotonic()) for r in range(self.world) if r != self.rank}
        while not self.stop.wait(self.period):
            try:
                self.beats += 1
                self.store.set(f"psoup/hb/{self.rank}", str(self.beats))
                if self.store.check([_ABORT_KEY]):
                    msg = self.store.get(_ABORT_KEY).decode(errors="replace")
                    if not self.stop.is_set():
                        self._abort(f"peer failure: {msg}")
                    return
                now = time.monotonic()
                for r in [r for r in seen if self.store.check([f"psoup/done/{r}"])]:
                    del seen[r]  # finished cleanly (shutdown): its heartbeat stops on purpose
                for r, (last, since) in seen.items():
                    key = f"psoup/hb/{r}"
                    cur = int(self.store.get(key)) if self.store.check([key]) else -1
                    if cur != last:
                        seen[r] = (cur, now)
                    elif now - since > self.peer_timeout and not self.stop.is_set():
                        try:
                            self.store.set(_ABORT_KEY, f"rank {r}: no heartbeat for {now - since:.0f} s")
                        except Exception:  # noqa: BLE001
                            pass
                        self._abort(f"peer failure: rank {r} stopped responding ({now - since:.0f} s without a "
                                    f"heartbeat)")
            except Exception as e:  # noqa: BLE001 - the store (rank 0's TCPStore) is gone
                if self.stop.is_set():
                    return
                self._abort(f"lost the rendezvous store ({type(e).__name__}: {e}); rank 0 has failed or exited")


def _start_watchdog(ctx: "DistContext") -> None:
    global _WATCHDOG
    if ctx.world_size <= 1 or os.environ.get("PSOUP_WATCHDOG", "1") == "0":
        return
    from torch.distributed import distributed_c10d

    store = distributed_c10d._get_default_store()
    period = float(os.environ.get("PSOUP_HEARTBEAT_S", "1.0"))
    peer_timeout = float(os.environ.get("PSOUP_PEER_TIMEOUT", "60"))
    store.set(f"psoup/hb/{ctx.rank}", "0")
    _WATCHDOG = _Watchdog(store, ctx.rank, ctx.world_size, period, peer_timeout)
    _WATCHDOG.start()


def report_failure(msg: str) -> None:
    """Publish this rank's failure so every peer aborts promptly (call before
    exiting non-zero).  Best effort: a dead store is not an error here."""
    ctx = _CTX
    if ctx is None or not ctx.distributed:
        return
    if _WATCHDOG is not None:
        _WATCHDOG.stop.set()  # this rank exits on its own
    try:
        from torch.distributed import distributed_c10d

        distributed_c10d._get_default_store().set(_ABORT_KEY, f"rank {ctx.rank}: {msg}")
    except Exception:  # noqa: BLE001
        pass


def peer_failure() -> Optional[str]:
    """The failure record a peer published ("rank r: msg"), or None.  A rank
    whose collective broke because a peer exited checks this first, so it
    reports the peer's failure, not the broken connection."""
    ctx = _CTX
    if ctx is None or not ctx.distributed:
        return None
    try:
        from torch.distributed import distributed_c10d

        store = distributed_c10d._get_default_store()
        if store.check([_ABORT_KEY]):
            return store.get(_ABORT_KEY).decode(errors="replace")
    except Exception:  # noqa: BLE001
        pass
    return None


def _peer_aware(fn):
    """A collective that breaks because a peer exited (gloo: "connection
    closed by peer") reports the peer's published failure, as the watchdog
    would a moment later, instead of the broken transport: the peer's record
    is waited for a few heartbeats before the original error is re-raised."""
    import functools

    @functools.wraps(fn)
    def wrapped(*args, **kwargs):
        try:
            return fn(*args, **kwargs)
        except Exception:
            ctx = _CTX
            if ctx is None or not ctx.distributed:
                raise
            period = float(os.environ.get("PSOUP_HEARTBEAT_S", "1.0"))
            deadline = time.monotonic() + max(1.0, 4 * period)
            while time.monotonic() < deadline:
                msg = peer_failure()
                if msg is not None:
                    if _WATCHDOG is not None:
                        _WATCHDOG.stop.set()
                        _WATCHDOG._abort(f"peer failure: {msg}")
                    sys.stderr.write(f"[rank {ctx.rank}] aborting: peer failure: {msg}\n")
                    sys.stderr.flush()
                    os._exit(3)
                time.sleep(0.05)
            raise

    return wrapped


def init(backend: Optional[str] = None, timeout_s: Optional[float] = None) -> DistContext:
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
    if timeout_s is None:
        # a last backstop only: peer death is caught by the heartbeat watchdog,
        # and collectives legitimately wait long (rank 0 reading a large
        # filterbank before the broadcast, shard imbalance before a gather)
        timeout_s = float(os.environ.get("PSOUP_COLLECTIVE_TIMEOUT", "1800"))
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
    if _CTX.distributed:
        _start_watchdog(_CTX)
    return _CTX


def context() -> DistContext:
    return _CTX if _CTX is not None else init()


def shutdown() -> None:
    global _CTX, _WATCHDOG
    if _WATCHDOG is not None:
        # peers may finish (and stop beating) before this rank: a clean
        # shutdown first marks this rank done (the peers' watches stop
        # expecting its heartbeat -- rank 0 may still be writing outputs long
        # after the others got here), then ends its own watch
        try:
            _WATCHDOG.store.set(f"psoup/done/{_WATCHDOG.rank}", "1")
        except Exception:  # noqa: BLE001 - the store is gone: the barrier below reports it
            pass
        _WATCHDOG.stop.set()
        _WATCHDOG.join(timeout=5)
        _WATCHDOG = None
        # every rank's watch has ended before rank 0 takes the store down
        barrier()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _CTX = None


@_peer_aware
def barrier() -> None:
    ctx = context()
    if ctx.distributed:
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


def _comm_device(ctx: DistContext) -> torch.device:
    return ctx.device if ctx.backend == "nccl" else torch.device("cpu")


@_peer_aware
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


@_peer_aware
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


@_peer_aware
def gather_buffers(payload: torch.Tensor, dst: int = 0, timing: Optional[dict] = None) -> Optional[List[torch.Tensor]]:
    """Variable-length gather of host uint8 tensors to ``dst`` only (sizes
    all-gathered, then one padded ``dist.gather``; RCCL on GPUs): the list of
    every rank's buffer (host tensors, rank order) on ``dst``, None elsewhere.
    Unlike :func:`gather_bytes` nothing reaches the other ranks and no Python
    ``bytes`` objects are made (candidate lists are tens of MB per rank).
    ``timing``: gets ``"sizes_done"`` (perf_counter after the size exchange,
    which is also where this rank waits for the slowest peer to arrive)."""
    ctx = context()
    assert payload.dtype == torch.uint8 and payload.dim() == 1
    if not ctx.distributed:
        return [payload]
    dev = _comm_device(ctx)
    n = torch.tensor([payload.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(ctx.world_size)]
    dist.all_gather(sizes, n)
    sizes_i = [int(s.item()) for s in sizes]
    if timing is not None:
        timing["sizes_done"] = time.perf_counter()
    mx = max(1, max(sizes_i))
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    if payload.numel():
        buf[: payload.numel()].copy_(payload)
    outs = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(ctx.world_size)] if ctx.rank == dst else None
    dist.gather(buf, outs, dst=dst)
    if ctx.rank != dst:
        return None
    return [o[:s].cpu() for o, s in zip(outs, sizes_i)]


@_peer_aware
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


@_peer_aware
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


@_peer_aware
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
    if total <= 0:
        return shard_range(n, world, rank)
    # item i goes to the shard its weight's midpoint falls in: contiguous,
    # and n equal items on n ranks are one each (a greedy cut at the first
    # item that reaches a rank's quota handed 86 + 85 trials to rank 0 and
    # none to rank 7 for 8 acceleration slices of 685 trials)
    owner = []
    acc = 0.0
    for x in w:
        owner.append(min(world - 1, int((acc + 0.5 * x) * world / total)))
        acc += x
    lo = next((i for i, o in enumerate(owner) if o >= rank), n)
    hi = next((i for i, o in enumerate(owner) if o > rank), n)
    return range(lo, hi)


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
