"""Multi-process collectives on the gloo backend (world_size 2, CPU)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

from peasoup_amd.parallel import dist as pdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch

        import peasoup_amd
        from peasoup_amd import _C

        ctx = pdist.init(backend="gloo")
        assert ctx.world_size == world and ctx.rank == rank
        # candidate gather: each rank serialises a different tree
        c = _C.Candidate(1.0 + rank, rank, 0.0, rank, 10.0 + rank, 2.0 + rank)
        c.assoc = [_C.Candidate(5.0, 7, 1.0, 1, 3.0, 4.0)] * (rank + 1)
        blobs = pdist.gather_bytes(_C.serialize_candidates([c]), dst=0)
        res = {}
        if rank == 0:
            got = [_C.deserialize_candidates(b)[0] for b in blobs]
            res["gather"] = [(g.dm_idx, g.count_assoc()) for g in got]
        # broadcast of a byte buffer (filterbank broadcast path)
        buf = torch.arange(1000, dtype=torch.int64).to(torch.uint8) if rank == 0 else None
        out = pdist.broadcast_bytes(buf, 1000)
        res["bcast"] = int(out.to(torch.int64).sum())
        s = pdist.broadcast_object_bytes(b"hello-header" if rank == 0 else None)
        res["obj"] = s
        t = torch.full((8,), rank + 1, dtype=torch.uint8)
        pdist.all_reduce_sum(t)
        res["allreduce"] = int(t[0])
        res["max"] = pdist.all_reduce_max_float(float(rank))
        pdist.barrier()
        q.put((rank, res))
        pdist.shutdown()
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_collectives(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
    assert out[0]["gather"] == [(r, r + 1) for r in range(world)]
    for r in range(world):
        assert out[r]["bcast"] == sum(i % 256 for i in range(1000))
        assert out[r]["obj"] == b"hello-header"
        assert out[r]["allreduce"] == world * (world + 1) // 2
        assert out[r]["max"] == float(world - 1)


def _queue_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import time

        pdist.init(backend="gloo")
        res = {}
        # two queues created in the same order on every rank: independent counters
        for name, n in (("dm", 40), ("dm", 7), ("other", 0)):
            wq = pdist.WorkQueue(name, n)
            mine = []
            while True:
                i = wq.claim()
                if i is None:
                    break
                mine.append(i)
                if rank == 0:
                    time.sleep(0.01)  # a slow rank: the others claim more
            res[f"{name}/{n}"] = mine
            pdist.barrier()
        q.put((rank, res))
        pdist.shutdown()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))


@pytest.mark.parametrize("world", [2, 3])
def test_work_queue_hands_out_each_index_once(world):
    """pdist.WorkQueue (the cross-rank DMDispenser): every index goes to
    exactly one rank, in increasing order per rank, and a slow rank gets fewer."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_queue_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
    for key, n in (("dm/40", 40), ("dm/7", 7), ("other/0", 0)):
        got = [i for r in range(world) for i in out[r][key]]
        assert sorted(got) == list(range(n)), key
        for r in range(world):
            assert out[r][key] == sorted(out[r][key])
    assert len(out[0]["dm/40"]) < 40 // world


def test_work_queue_without_process_group():
    wq = pdist.WorkQueue("local-test", 3)
    assert [wq.claim() for _ in range(5)] == [0, 1, 2, None, None]
    assert wq.claimed == [0, 1, 2]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partitions(world):
    n = 59
    shards = [pdist.shard_range(n, world, r) for r in range(world)]
    assert sum(len(s) for s in shards) == n
    assert [i for s in shards for i in s] == list(range(n))
    w = [1.0 + (i % 7) for i in range(n)]
    shards = [pdist.shard_range(n, world, r, w) for r in range(world)]
    assert [i for s in shards for i in s] == list(range(n))
    loads = [sum(w[i] for i in s) for s in shards]
    assert max(loads) - min(loads) <= max(w) + 1e-9


def _timeshard_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import numpy as np
        import torch

        from peasoup_amd import _C
        from peasoup_amd.parallel import timeshard
        from peasoup_amd.utils import reference as ref
        from peasoup_amd.utils import sigproc, synthetic

        pdist.init(backend="gloo")
        nchans, nbits, nsamps = 32, 2, 3000
        hdr = synthetic.make_header(nchans=nchans, nbits=nbits, tsamp=0.00032, fch1=1510.0, foff=-2.0,
                                    nsamples=nsamps)
        dms = _C.generate_dm_list(0.0, 120.0, 0.00032, 64.0, 1510.0, -2.0, nchans, 1.1)
        vals = np.random.default_rng(5).integers(0, 4, size=(nsamps, nchans), dtype=np.uint8)
        packed = sigproc.pack_samples(vals, nbits)
        plan = timeshard.make_plan(hdr, nsamps, dms, world)
        own = torch.from_numpy(timeshard.slice_packed(packed, plan, rank).copy())
        mine = timeshard.time_sharded_dedisperse(own, plan, timeshard.reference_dedisperser(hdr, dms))
        offs = ref.dm_offsets(dms, ref.delay_table(nchans, 0.00032, 1510.0, -2.0))
        full = ref.dedisperse(vals, offs, nbits, None, plan.out_nsamps)
        s = plan.dm_shards[rank]
        q.put((rank, {"ok": bool(np.array_equal(mine.numpy(), full[s.start:s.stop])), "shape": tuple(mine.shape),
                      "max_delay": plan.max_delay}))
        pdist.shutdown()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, {"error": traceback.format_exc()}))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_time_sharded_dedispersion_gloo(world):
    """Halo exchange + all-to-all corner turn == whole-observation dedispersion."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeshard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
        assert out[r]["ok"], out[r]
    assert out[0]["max_delay"] > 0
