"""Asynchronous point-to-point record links (the split topology's transport).

Reference: actors never wait for the learner -- they pickle experience into files and go on
acting; the learner picks the files up whenever it polls (``/root/reference/actor.py:64-66``,
``learner.py:53-66``, ``replay_memory.py:125-173``).  A lock-step exchange (every learner blocks
in ``recv`` on every feeding actor, every actor in ``send``) lets one slow actor rank stall its
learner and, through the data-parallel all-reduce, every learner.  These links restore the
decoupling over ``torch.distributed``:

* a **payload** (a fixed-size uint8 record or a weight snapshot) travels on the data group --
  RCCL over xGMI between GPUs (device buffers, the bytes never visit the host), gloo in CPU tests;
* the **control plane** is two counters per link in the job's c10d store (``sent``, ``taken``):
  the sender bumps ``sent`` and posts its ``isend``; the receiver reads ``sent`` when it polls
  (one store round trip per source) and posts a payload ``recv`` only for messages already sent,
  so a receiver never waits on a peer and a GPU receiver never has an RCCL kernel parked on its
  chip while its persistent kernels run; ``taken`` tells the sender how many slots are free;
* a sender owns ``slots`` payload buffers and blocks only when every one is still untaken.
  Before a buffer is refilled its send ``Work`` is waited: a CPU wait for gloo, a stream wait
  for RCCL (the refilling kernel is ordered after the send; the host does not block).

(gloo's point-to-point ``Work.is_completed()`` stays False until ``wait()`` is called, so
completion cannot be polled on the work objects themselves -- hence the store counters.)

Payloads of one link travel in order (same src / dst / tag), so per-link order and loss-freedom
follow from the counters; record payloads also carry their own sequence numbers, which the
consumers check.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist


def _store():
    return dist.distributed_c10d._get_default_store()


def _count(store, key: str) -> int:
    return int(store.add(key, 0))


class LinkSender:
    """Sender side of the link ``name`` to ``dst``: ``slots`` payload buffers of ``nbytes``
    (device or host).  ``acquire()`` returns the next free buffer (blocking only while all are
    untaken), ``send()`` ships it."""

    def __init__(self, name: str, dst: int, nbytes: int, slots: int, device, data_group=None,
                 tag: int = 0, host_stage: bool = False):
        self.key, self.dst, self.nbytes, self.slots = name, int(dst), int(nbytes), int(slots)
        self.data, self.tag = data_group, int(tag)
        self.store = _store()
        self.device = torch.device(device)
        self.bufs = [self._alloc() for _ in range(self.slots)]
        # gloo payloads travel from host memory: a pinned staging copy per slot
        self.host = [torch.empty(self.nbytes, dtype=torch.uint8,
                                 pin_memory=self.device.type == "cuda") for _ in range(self.slots)] \
            if host_stage else None
        self.works: List[Optional[object]] = [None] * self.slots
        self.seq = 0
        self.taken = 0
        self.stalls = 0          # acquire() calls that found every slot untaken
        self.stall_s = 0.0

    def _alloc(self) -> torch.Tensor:
        buf = torch.zeros(self.nbytes + 64, dtype=torch.uint8, device=self.device)
        off = (-buf.data_ptr()) % 64
        return buf[off: off + self.nbytes]

    def refresh(self) -> int:
        self.taken = _count(self.store, self.key + "/taken")
        return self.taken

    def in_flight(self, refresh: bool = True) -> int:
        if refresh:
            self.refresh()
        return self.seq - self.taken

    def acquire(self) -> torch.Tensor:
        if self.seq - self.taken >= self.slots and self.in_flight() >= self.slots:
            self.stalls += 1
            t0 = time.perf_counter()
            while self.in_flight() >= self.slots:
                time.sleep(0.0002)
            self.stall_s += time.perf_counter() - t0
        q = self.seq % self.slots
        if self.works[q] is not None:
            self.works[q].wait()       # gloo: returns at once (taken); RCCL: stream order
            self.works[q] = None
        return self.bufs[q]

    def send(self) -> None:
        """Ship the buffer last returned by ``acquire``.  ``sent`` is bumped before the isend: a
        first RCCL send between two ranks blocks in the communicator set-up until the receiver
        joins, which it does once it has seen the count."""
        q = self.seq % self.slots
        payload = self.bufs[q]
        if self.host is not None:
            self.host[q].copy_(payload)
            payload = self.host[q]
        self.seq += 1
        self.store.add(self.key + "/sent", 1)
        self.works[q] = dist.isend(payload, self.dst, group=self.data, tag=self.tag)

    def flush(self, timeout_s: float = 600.0) -> None:
        """Block until every sent payload has been taken."""
        t0 = time.perf_counter()
        while self.in_flight() > 0:
            time.sleep(0.0005)
            if time.perf_counter() - t0 > timeout_s:
                raise TimeoutError(f"link {self.key}: {self.in_flight()} payloads never taken")
        for q in range(self.slots):
            if self.works[q] is not None:
                self.works[q].wait()
                self.works[q] = None

    def close(self) -> None:
        """Mark the link finished (after the last send); the receiver's ``wait_closed`` returns
        once it has taken everything."""
        self.store.add(self.key + "/closed", 1)


class LinkReceiver:
    """Receiver side of the links ``names[i]`` from ``srcs[i]``: ``poll()`` takes every message
    already sent (payload ``recv`` into the per-link buffer, then ``on_message(i, buf)``) and never
    waits for a link on which nothing was sent."""

    def __init__(self, names: List[str], srcs: List[int], nbytes: int, device, on_message: Callable,
                 data_group=None, tag: int = 0, host_stage: bool = False):
        self.keys, self.srcs = list(names), list(srcs)
        self.nbytes, self.data, self.tag = int(nbytes), data_group, int(tag)
        self.store = _store()
        self.device = torch.device(device)
        self.on_message = on_message
        self.bufs = []
        for _ in self.srcs:
            b = torch.zeros(self.nbytes + 64, dtype=torch.uint8, device=self.device)
            off = (-b.data_ptr()) % 64
            self.bufs.append(b[off: off + self.nbytes])
        self.host = [torch.empty(self.nbytes, dtype=torch.uint8) for _ in self.srcs] if host_stage else None
        self.received = [0] * len(self.srcs)
        self.last_poll = 0.0

    def _take(self, i: int) -> None:
        if self.host is not None:
            dist.recv(self.host[i], self.srcs[i], group=self.data, tag=self.tag)
            self.bufs[i].copy_(self.host[i], non_blocking=True)
        else:
            # RCCL: enqueued on the communication stream behind the current stream's work, and
            # the current stream waits for it -- ordered between the learner's graph replays
            dist.recv(self.bufs[i], self.srcs[i], group=self.data, tag=self.tag)
        self.received[i] += 1
        self.on_message(i, self.bufs[i])
        self.store.add(self.keys[i] + "/taken", 1)

    def poll(self, max_per_link: int = 1 << 30, min_interval_s: float = 0.0) -> int:
        """Take the messages already sent (at most ``max_per_link`` per link); never waits."""
        now = time.perf_counter()
        if now - self.last_poll < min_interval_s:
            return 0
        self.last_poll = now
        n = 0
        for i in range(len(self.srcs)):
            avail = _count(self.store, self.keys[i] + "/sent") - self.received[i]
            for _ in range(min(avail, max_per_link)):
                self._take(i)
                n += 1
        return n

    def wait_for(self, counts: Dict[int, int], timeout_s: float = 600.0) -> None:
        """Block until link i has delivered ``counts[i]`` messages (the drain at the end)."""
        t0 = time.perf_counter()
        while any(self.received[i] < c for i, c in counts.items()):
            if self.poll() == 0:
                time.sleep(0.0005)
            if time.perf_counter() - t0 > timeout_s:
                raise TimeoutError(f"links {self.keys}: received {self.received}, expected {counts}")

    def wait_closed(self, timeout_s: float = 600.0) -> None:
        """Take messages until every link is closed and drained."""
        t0 = time.perf_counter()
        while True:
            self.poll()
            closed = all(_count(self.store, k + "/closed") > 0 for k in self.keys)
            if closed and self.poll() == 0 and all(
                    _count(self.store, k + "/sent") == r for k, r in zip(self.keys, self.received)):
                return
            time.sleep(0.0005)
            if time.perf_counter() - t0 > timeout_s:
                raise TimeoutError(f"links {self.keys}: not closed after {timeout_s} s")
