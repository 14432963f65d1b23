"""Timers and roctx ranges (reference: include/utils/stopwatch.hpp,
include/utils/nvtx.hpp -> rocprofv3 --marker-trace ranges)."""
from __future__ import annotations

import contextlib
import time


class Stopwatch:
    """Accumulating wall-clock timer; ``get_time()`` returns seconds."""

    def __init__(self) -> None:
        self._acc = 0.0
        self._t0 = None

    def start(self) -> None:
        self._t0 = time.perf_counter()

    def stop(self) -> None:
        if self._t0 is not None:
            self._acc += time.perf_counter() - self._t0
            self._t0 = None

    def add(self, seconds: float) -> None:
        """Accumulate an externally measured interval (e.g. GPU event time)."""
        self._acc += float(seconds)

    def reset(self) -> None:
        self._acc = 0.0
        self._t0 = None

    def get_time(self) -> float:
        t = self._acc
        if self._t0 is not None:
            t += time.perf_counter() - self._t0
        return t


@contextlib.contextmanager
def roctx_range(name: str):
    """roctx push/pop around a block (visible with rocprofv3 --marker-trace)."""
    from .. import _C

    _C.roctx_push(name)
    try:
        yield
    finally:
        _C.roctx_pop()


class GpuTimer:
    """hipEvent-based interval timer on the current stream (milliseconds)."""

    def __init__(self) -> None:
        import torch

        self._a = torch.cuda.Event(enable_timing=True)
        self._b = torch.cuda.Event(enable_timing=True)

    def start(self) -> None:
        self._a.record()

    def stop(self) -> float:
        self._b.record()
        self._b.synchronize()
        return self._a.elapsed_time(self._b)
