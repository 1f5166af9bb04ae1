"""Tracing / profiling (the reference has none).

* ``roctx_range(name)`` -- ROCTx ranges (``libroctx64``, shipped with ROCm and torch) around
  learner/actor phases; visible in ``rocprofv3 --marker-trace`` timelines.  No-op when the
  library is absent.
* ``PhaseTimer`` -- HIP-event timing of named phases on the current stream (no host sync until
  ``summary()``), used by ``bench.py --profile-phases`` and the metrics stream.
* ``torch_profiler(...)`` -- thin wrapper over torch.profiler with ROCm (CUDA) activities.
"""
from __future__ import annotations

import contextlib
import ctypes
import glob
import os
from collections import defaultdict
from typing import Dict, List, Optional

import torch

_roctx = None
_roctx_tried = False


def _load_roctx():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so")]
    cands += glob.glob("/opt/rocm/lib/libroctx64.so*")
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            break
        except (OSError, AttributeError):
            continue
    return _roctx


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _load_roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def roctx_mark(name: str) -> None:
    lib = _load_roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class PhaseTimer:
    """Accumulate GPU time per phase with events; ``summary()`` synchronises once."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._pending: List = []
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            with roctx_range(name):
                yield
            return
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        with roctx_range(name):
            yield
        b.record()
        self._pending.append((name, a, b))

    def summary(self) -> Dict[str, float]:
        if self._pending:
            torch.cuda.synchronize()
            for name, a, b in self._pending:
                self.totals[name] += a.elapsed_time(b)
                self.counts[name] += 1
            self._pending.clear()
        return {k: v / max(self.counts[k], 1) for k, v in self.totals.items()}


def torch_profiler(trace_dir: Optional[str] = None, **kw):
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    handler = torch.profiler.tensorboard_trace_handler(trace_dir) if trace_dir else None
    return torch.profiler.profile(activities=acts, on_trace_ready=handler, **kw)
