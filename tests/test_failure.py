"""Peer-failure handling, CPU / gloo world 3: a rank that
fails publishes its failure and every peer aborts with rank context within
seconds instead of blocking in a collective; a peer killed without reporting
is detected by its stale heartbeat; a clean run exits 0 on every rank."""
import os
import signal
import socket
import subprocess
import sys
import time

from conftest import REPO

WORLD = 3

SCRIPT = r"""
import os, sys, time
sys.path.insert(0, %r)
from peasoup_amd.parallel import dist as pdist
mode = sys.argv[1]
ctx = pdist.init(backend="gloo")
import torch
t = torch.ones(4)
pdist.all_reduce_sum(t)
print(f"rank {ctx.rank} ready", flush=True)
if ctx.rank == 1 and mode == "raise":
    time.sleep(1.0)
    try:
        raise RuntimeError("fault injection: rank 1 aborting")
    except RuntimeError as e:
        print(f"[rank 1] peasoup failed: {e}", file=sys.stderr, flush=True)
        pdist.report_failure(str(e))
        os._exit(1)
if ctx.rank == 1 and mode == "hang":
    import signal
    os.kill(os.getpid(), signal.SIGSTOP)  # frozen: alive to the transport, silent to the watchdog
if mode == "clean":
    time.sleep(0.5 * ctx.rank)  # ranks finish at different times
    pdist.all_reduce_sum(t)
    pdist.shutdown()
    sys.exit(0)
if mode == "slowroot":
    # the others are done; rank 0 keeps working (writing outputs) for longer
    # than the peer timeout with its watchdog live, then shuts down
    if ctx.rank == 0:
        time.sleep(float(os.environ["PSOUP_PEER_TIMEOUT"]) * 2.5)
    pdist.shutdown()
    sys.exit(0)
pdist.barrier()  # rank 1 never arrives
print("barrier passed", flush=True)
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, mode, extra_env=None, limit=90, skip=()):
    f = tmp_path / "w.py"
    f.write_text(SCRIPT % REPO)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(WORLD),
               PSOUP_HEARTBEAT_S="0.2", PSOUP_COLLECTIVE_TIMEOUT="600", **(extra_env or {}))
    t0 = time.monotonic()
    procs = [subprocess.Popen([sys.executable, str(f), mode], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
             for r in range(WORLD)]
    res = [None] * WORLD
    try:
        for r in [q for q in range(WORLD) if q not in skip] + list(skip):
            p = procs[r]
            if r in skip:
                os.killpg(p.pid, signal.SIGKILL)
            out, err = p.communicate(timeout=limit)
            res[r] = (p.returncode, out, err)
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
    return res, time.monotonic() - t0


def test_failing_rank_aborts_every_peer(tmp_path):
    res, dt = _run(tmp_path, "raise")
    assert dt < 60, dt
    for r, (rc, out, err) in enumerate(res):
        assert rc != 0, (r, out, err)
        assert "barrier passed" not in out
        assert "rank 1" in err, (r, err[-2000:])
    assert "[rank 0] aborting: peer failure: rank 1: fault injection" in res[0][2]
    assert "[rank 2] aborting: peer failure: rank 1: fault injection" in res[2][2]


def test_silent_rank_is_detected_by_heartbeat(tmp_path):
    """Rank 1 stops (SIGSTOP) without reporting: its transport stays open, so
    the collective alone would block until the process-group timeout; the
    peers see its heartbeat stall and abort."""
    res, dt = _run(tmp_path, "hang", {"PSOUP_PEER_TIMEOUT": "4"}, skip=(1,))
    assert dt < 60, dt
    for r in (0, 2):
        rc, out, err = res[r]
        assert rc == 3, (r, rc, err[-2000:])
        assert "aborting: peer failure: rank 1" in err, err[-2000:]


def test_clean_run_exits_zero(tmp_path):
    res, _ = _run(tmp_path, "clean", {"PSOUP_PEER_TIMEOUT": "4"})
    for r, (rc, out, err) in enumerate(res):
        assert rc == 0, (r, err[-2000:])
        assert "aborting" not in err


def test_slow_root_after_peers_finish_exits_zero(tmp_path):
    """Peers that reached shutdown() stop beating on purpose: rank 0, still
    busy past PSOUP_PEER_TIMEOUT with its watchdog running, must not declare
    them dead (a false abort before the outputs are written)."""
    res, dt = _run(tmp_path, "slowroot", {"PSOUP_PEER_TIMEOUT": "2"})
    for r, (rc, out, err) in enumerate(res):
        assert rc == 0, (r, rc, err[-2000:])
        assert "aborting" not in err
