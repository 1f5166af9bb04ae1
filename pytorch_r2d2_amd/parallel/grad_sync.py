"""Data-parallel gradient synchronisation for the flat gradient buffer.

The learner's gradients live in ONE flat fp32 buffer (engine/layout.py) split into two
buckets in backward-completion order:

    core  = LSTM + dueling head (~99% of the 8.15 MB; complete right after BPTT + weight GEMMs)
    torso = conv weights (complete last)

``GradSync.start(lo, hi)`` launches an all-reduce of a bucket on a dedicated communication
stream after an event recorded on the compute stream, so the 8 MB core all-reduce over xGMI
overlaps the conv backward; ``finish()`` makes the compute stream wait for all outstanding
buckets before the optimizer.  Optional bf16 compression halves the bytes on the wire (the
sum is accumulated by RCCL in bf16; the result is written back to fp32).

Sizing for MI355X xGMI (7 links x ~153 GB/s per GPU): at 8 ranks a ring all-reduce of 8 MB
moves 2*(7/8)*8 MB per GPU -> ~15 us when RCCL stripes all links, ~93 us single-ring; either is
hidden under the ~100+ us conv backward.  More, smaller buckets would only add latency.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class GradSync:
    def __init__(self, grad: torch.Tensor, world: int, group=None, dtype: str = "fp32",
                 use_stream: bool = True, force: bool = False):
        self.grad = grad
        self.world = world
        self.force = force            # issue the collectives at world 1 too (dist.force_dp)
        self.group = group
        self.dtype = dtype
        self.cuda = grad.is_cuda
        self.stream = torch.cuda.Stream(device=grad.device) if (self.cuda and use_stream) else None
        self._pending: List = []
        self._bufs = {}

    def start(self, lo: int, hi: int) -> None:
        if (self.world <= 1 and not self.force) or hi <= lo:
            return
        view = self.grad[lo:hi]
        if self.stream is None:
            self._reduce(view, lo)
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.grad.device))
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            self._reduce(view, lo)
            done = torch.cuda.Event()
            done.record(self.stream)
        self._pending.append(done)

    def _reduce(self, view: torch.Tensor, key: int) -> None:
        if self.dtype == "bf16":
            buf = self._bufs.get(key)
            if buf is None or buf.numel() != view.numel():
                buf = torch.empty(view.numel(), dtype=torch.bfloat16, device=view.device)
                self._bufs[key] = buf
            buf.copy_(view)
            dist.all_reduce(buf, group=self.group)
            view.copy_(buf)
        else:
            dist.all_reduce(view, group=self.group)

    def finish(self) -> None:
        if not self._pending:
            return
        cur = torch.cuda.current_stream(self.grad.device)
        for ev in self._pending:
            cur.wait_event(ev)
        self._pending.clear()


def allreduce_mean_(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    if world > 1:
        dist.all_reduce(t, group=group)
        t.div_(world)
    return t
