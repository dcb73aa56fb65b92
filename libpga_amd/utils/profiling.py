"""Tracing and timing helpers (SURVEY.md §5.1 — the reference has none).

* ``trace_range(name)``: a roctx range (visible to ``rocprofv3
  --marker-trace``) when ``PGA_TRACE`` >= 1; a no-op otherwise.  The native
  engine marks its own stages (csrc/engine/trace.cpp).
* ``GpuTimer``: HIP-event timing on the current stream (host clock on CPU).
"""
from __future__ import annotations

import contextlib
import time
from typing import Iterator, Optional

import torch

from .._ext import C


def tracing_enabled() -> bool:
    return C.trace_level() > 0


@contextlib.contextmanager
def trace_range(name: str) -> Iterator[None]:
    if C.trace_level() > 0:
        C.trace_push(name)
        try:
            yield
        finally:
            C.trace_pop()
    else:
        yield


def trace_mark(name: str) -> None:
    C.trace_mark(name)


class GpuTimer:
    """``with GpuTimer(device) as t: ...`` then ``t.ms``.

    On a GPU the interval is measured between two HIP events recorded on the
    current stream (so it covers exactly the enqueued work); on the CPU it is
    the wall clock."""

    def __init__(self, device: Optional[torch.device] = None):
        self.device = torch.device(device) if device is not None else None
        self.ms = 0.0

    def _gpu(self) -> bool:
        return self.device is not None and self.device.type == "cuda"

    def __enter__(self) -> "GpuTimer":
        if self._gpu():
            self._a = torch.cuda.Event(enable_timing=True)
            self._b = torch.cuda.Event(enable_timing=True)
            self._a.record(torch.cuda.current_stream(self.device))
        else:
            self._t = time.perf_counter()
        return self

    def __exit__(self, *exc) -> None:
        if self._gpu():
            self._b.record(torch.cuda.current_stream(self.device))
            self._b.synchronize()
            self.ms = self._a.elapsed_time(self._b)
        else:
            self.ms = (time.perf_counter() - self._t) * 1e3
