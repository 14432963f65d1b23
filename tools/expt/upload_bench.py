"""Host -> device upload paths for a page-cached filterbank-sized file (the
native setup's load_filterbank_fanout cost): mmap + pageable copy, read() +
pageable copy, pread into pinned chunks, host-register of the mapping."""
import mmap
import os
import sys
import time

import numpy as np
import torch

path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/upload_bench.bin"
nbytes = 268 << 20
if not os.path.exists(path) or os.path.getsize(path) != nbytes:
    with open(path, "wb") as f:
        f.write(np.random.default_rng(0).integers(0, 256, nbytes, dtype=np.uint8).tobytes())
with open(path, "rb") as f:  # page cache warm
    while f.read(64 << 20):
        pass
dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()


def t(name, fn, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"{name:40s} " + " ".join(f"{1e3 * x:7.1f}" for x in ts) + " ms", flush=True)


def mmap_copy():
    with open(path, "rb") as f:
        m = mmap.mmap(f.fileno(), 0, prot=mmap.PROT_READ)
        dev.copy_(torch.frombuffer(m, dtype=torch.uint8))
        m.close()


def read_copy():
    a = np.fromfile(path, dtype=np.uint8)
    dev.copy_(torch.from_numpy(a))


def pinned_alloc(mb):
    return lambda: torch.empty(mb << 20, dtype=torch.uint8, pin_memory=True)


def pread_pinned(chunk_mb, nthreads=1):
    from concurrent.futures import ThreadPoolExecutor

    stage = [torch.empty(chunk_mb << 20, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    ev = [torch.cuda.Event(), torch.cuda.Event()]
    pool = ThreadPoolExecutor(nthreads)

    def run():
        fd = os.open(path, os.O_RDONLY)
        ch = chunk_mb << 20
        used = [False, False]
        s = torch.cuda.current_stream()
        for k, off in enumerate(range(0, nbytes, ch)):
            j = k & 1
            if used[j]:
                ev[j].synchronize()
            n = min(ch, nbytes - off)
            mv = memoryview(stage[j].numpy())
            part = (n + nthreads - 1) // nthreads
            list(pool.map(lambda i: os.preadv(fd, [mv[i * part:min(n, (i + 1) * part)]], off + i * part),
                          range(nthreads)))
            dev[off:off + n].copy_(stage[j][:n], non_blocking=True)
            ev[j].record(s)
            used[j] = True
        os.close(fd)

    return run


t("mmap -> device (pageable)", mmap_copy)
t("read -> device (pageable)", read_copy)
t("pinned alloc 16 MB", pinned_alloc(16))
t("pinned alloc 64 MB", pinned_alloc(64))
t("pinned alloc 268 MB", pinned_alloc(268))
for ch, th in ((16, 1), (16, 4), (32, 4), (64, 4), (64, 8)):
    t(f"pread {ch} MB pinned x2, {th} threads", pread_pinned(ch, th))
