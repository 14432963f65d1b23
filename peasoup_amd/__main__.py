"""``python -m peasoup_amd [peasoup flags]`` (or ``python -m peasoup_amd ffa
[ffaster flags]`` for the FFA search) -- the peasoup CLI as a
torchrun-compatible, one-process-per-GPU program:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m peasoup_amd -i obs.fil --dm_end 1000 --acc_start -500 --acc_end 500 -n 3 --npdmp 128

Flags are identical to the native ``bin/peasoup`` (include/utils/cmdline.hpp).
A single process uses one GPU; the native CLI's ``-t`` thread-per-GPU mode
remains available in ``bin/peasoup``.

Failure handling: a failing rank prints its error with its
rank and exits immediately, so torchrun tears the group down instead of
letting the peers hang in a collective.  Elastic recovery is torchrun's
restart plus resume:

    python -m torch.distributed.run --max-restarts 3 ... -m peasoup_amd ... --checkpoint_dir ck/

re-runs the group after a failure and every rank skips the DM chunks whose
spill files (``ck/dm_<d0>_<d1>.psoc``) already exist.
"""
from __future__ import annotations

import sys


def _fail_hard(what: str, e: BaseException) -> None:
    """A failed rank must not leave its peers blocked in a collective: report
    with rank context and exit hard, which destroys this rank's RCCL
    communicator (the ncclCommAbort equivalent) and makes torchrun stop -- or,
    with --max-restarts, restart -- the worker group (a restart with
    --checkpoint_dir resumes from the per-DM spill files).  When a peer failed
    first (this rank's collective broke with it), the peer's record is
    reported instead of the broken connection."""
    import os
    import traceback

    from .parallel import dist as pdist

    rank = os.environ.get("RANK", "0")
    peer = pdist.peer_failure()
    if peer is not None:
        print(f"[rank {rank}] aborting: peer failure: {peer}", file=sys.stderr)
        sys.stderr.flush()
        if rank == "0":
            import time

            time.sleep(2.0)  # rank 0 hosts the store: let the other peers read the record
        os._exit(3)
    print(f"[rank {rank}] {what} failed: {e}", file=sys.stderr)
    pdist.report_failure(f"{type(e).__name__}: {e}")
    traceback.print_exc()
    sys.stderr.flush()
    sys.stdout.flush()
    os._exit(1)


def main(argv=None) -> int:
    from . import _C
    from .models.search import run_search
    from .parallel import dist as pdist

    argv = list(sys.argv if argv is None else argv)
    if len(argv) > 1 and argv[1] == "ffa":
        return _main_ffa(["ffaster"] + argv[2:])
    argv[0] = "peasoup"
    ok, exit_now, args = _C.parse_cmdline(argv)
    if not ok:
        print("Failed to parse command line arguments.", file=sys.stderr)
        return 1
    if exit_now:
        return 0
    if args.verbose:
        _C.set_log_level(2)
    try:
        res = run_search(args)
    except BaseException as e:  # noqa: BLE001 - any failure must tear the job down
        _fail_hard("peasoup", e)
    if res is not None and (args.verbose or args.progress_bar):
        print(f"Wrote {len(res.candidates)} candidates to {args.outdir}; "
              f"{res.performance['dm_accel_trials_per_sec']:.1f} DMxaccel trials/s over {int(res.performance['ranks'])} rank(s)")
    pdist.shutdown()
    return 0


def _main_ffa(argv) -> int:
    from . import _C
    from .models.ffa import run_ffa_search
    from .parallel import dist as pdist

    ok, exit_now, args = _C.parse_ffa_cmdline(argv)
    if not ok:
        print("Failed to parse command line arguments.", file=sys.stderr)
        return 1
    if exit_now:
        return 0
    try:
        res = run_ffa_search(args)
    except BaseException as e:  # noqa: BLE001 - same teardown policy as the search
        _fail_hard("ffa", e)
    if res is not None and args.verbose:
        print(f"Wrote {len(res.candidates)} FFA candidates to {args.outfilename}")
    pdist.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
