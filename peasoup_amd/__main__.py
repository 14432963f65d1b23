"""``python -m peasoup_amd [peasoup flags]`` -- the peasoup CLI as a
torchrun-compatible, one-process-per-GPU program:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m peasoup_amd -i obs.fil --dm_end 1000 --acc_start -500 --acc_end 500 -n 3 --npdmp 128

Flags are identical to the native ``bin/peasoup`` (include/utils/cmdline.hpp).
A single process uses one GPU; the native CLI's ``-t`` thread-per-GPU mode
remains available in ``bin/peasoup``.
"""
from __future__ import annotations

import sys


def main(argv=None) -> int:
    from . import _C
    from .models.search import run_search
    from .parallel import dist as pdist

    argv = list(sys.argv if argv is None else argv)
    argv[0] = "peasoup"
    ok, exit_now, args = _C.parse_cmdline(argv)
    if not ok:
        print("Failed to parse command line arguments.", file=sys.stderr)
        return 1
    if exit_now:
        return 0
    if args.verbose:
        _C.set_log_level(2)
    res = run_search(args)
    if res is not None and (args.verbose or args.progress_bar):
        print(f"Wrote {len(res.candidates)} candidates to {args.outdir}; "
              f"{res.performance['dm_accel_trials_per_sec']:.1f} DMxaccel trials/s over {int(res.performance['ranks'])} rank(s)")
    pdist.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
