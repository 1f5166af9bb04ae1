"""CPU actors -> HBM replay: the native trajectory ingest (BASELINE config 2).

Reference: every actor pickles its 50k-row local replay to ``memory{id}.pt`` every 5 episodes
and the learner polls the files every 20 steps, unpickles them (1.23 s per 5k rows, 233 MB) and
numpy-copies them into its host ring (``replay_memory.py:125-173``, ``learner.py:111-116``).

Here each CPU actor process owns one shared-memory SPSC ring (``runtime.ShmRing``) and pushes its
local replay as ONE packed record (``parallel.trajectory.pack_rows``: header + SoA fields at
64-byte aligned offsets).  The learner process, between its graph-replayed steps:

1. takes the front record of each ring **zero-copy** (``ShmRing.front``),
2. DMAs it to a device staging buffer with ``hipMemcpyAsync`` on a copy stream -- straight from
   the ring when the ring mapping could be registered with the HIP runtime
   (``hipHostRegister``), else through a pinned bounce buffer,
3. makes the learner stream wait for that copy and launches the device ingest
   (``csrc/kernels/ingest.hip``: the record is parsed on the device, rows scattered into the
   actor's sub-ring at a device-side write head, start flags / leaves / n_valid updated, changed
   leaves appended to the dirty list),
4. repairs the sum tree from the dirty list -- a full rebuild once the poll's records together
   could overflow half the dirty list (every record of a poll appends to the same list before
   the one repair at its end),
5. releases the ring bytes once the DMA has completed (event query, never a blocking sync on
   the learner stream).

Nothing here reads device memory back to the host.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np
import torch

from ..ops._lib import check, kernels, ptr, stream_handle
from ..parallel.trajectory import ShmTrajectoryReader, header_bytes, validate_record

_VP = ctypes.c_void_p


class IngestArgs(ctypes.Structure):
    """Mirror of ``struct IngestArgs`` (csrc/kernels/ingest.hip); size checked against the .so."""
    _fields_ = [("rec", _VP), ("rec_bytes", ctypes.c_longlong), ("sub", ctypes.c_int),
                ("max_rows", ctypes.c_int)] + [
        (n, _VP) for n in ("ihead", "rows_total", "err", "frames", "hs_cs", "ths_cs", "action",
                           "reward", "done", "priority", "is_start", "leaves", "n_valid", "dirty",
                           "count")] + [
        (n, ctypes.c_int) for n in ("max_dirty", "FB", "H2", "cap_e", "rows_per_sub", "start_lag",
                                    "n_sub", "pad_")]


def ingest_args(replay, rec: int, rec_bytes: int, sub: int, use_dirty: bool,
                rows_per_sub: int = 0, start_lag: int = 0) -> IngestArgs:
    """``rows_per_sub`` > 0: the record is env-major blocks of that many rows, block i to sub-ring
    ``sub + i``; ``start_lag``: its start column marks the position ``start_lag`` rows before each
    row (an actor rank's blocks, parallel/actor_ranks.py).  The device rejects (error word) a
    record that is not whole blocks or addresses sub-rings past the replay's."""
    if ctypes.sizeof(IngestArgs) != kernels().r2_ingest_args_bytes():
        raise RuntimeError("IngestArgs layout differs from csrc/kernels/ingest.hip")
    rp = replay
    a = IngestArgs()
    a.rec, a.rec_bytes, a.sub = rec, int(rec_bytes), int(sub)
    a.max_rows = int(min(rp.cap_e, rec_bytes // max(rp.frame_bytes, 1) + 1))
    for name, t in (("ihead", rp.ihead), ("rows_total", rp.rows_total_d), ("err", rp.ingest_err),
                    ("frames", rp.frames), ("hs_cs", rp.hs_cs), ("ths_cs", rp.target_hs_cs),
                    ("action", rp.action), ("reward", rp.reward), ("done", rp.done),
                    ("priority", rp.priority), ("is_start", rp.is_start), ("leaves", rp.tree),
                    ("n_valid", rp.n_valid), ("count", rp.dirty_count)):
        setattr(a, name, ptr(t))
    a.dirty = ptr(rp.dirty) if use_dirty else 0
    a.max_dirty, a.FB, a.H2, a.cap_e = rp.max_dirty, rp.frame_bytes, 2 * rp.H, rp.cap_e
    a.rows_per_sub, a.start_lag, a.n_sub = int(rows_per_sub), int(start_lag), rp.n_sub
    if rows_per_sub > 0:   # env-major windows: every row of the record is kept
        a.max_rows = int(rec_bytes // max(rp.frame_bytes, 1) + 1)
    return a


class HBMIngestor:
    """Learner-side consumer of N CPU-actor shared-memory rings (actor i -> sub-ring i)."""

    def __init__(self, replay, ring_names: List[str], ring_bytes: int = 256 << 20,
                 register: bool = True, stream=None):
        self.rp = replay
        if replay.n_sub < len(ring_names):
            raise ValueError("one HBM sub-ring per actor ring")
        self.readers = [ShmTrajectoryReader(n, ring_bytes) for n in ring_names]
        dev = replay.device
        self.copy_stream = torch.cuda.Stream(device=dev)
        self.stream = stream            # learner stream (None: current stream at poll time)
        self.dev_buf = [torch.empty(0, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.dev_done = [torch.cuda.Event() for _ in range(2)]
        self.slot = 0
        # zero-copy DMA source: register every ring mapping with the HIP runtime
        self.registered = []
        for r in self.readers:
            base, size = r.ring.mapping()
            ok = register and kernels().r2_host_register(_VP(base), size) == 0
            self.registered.append(base if ok else None)
        self.pinned = None
        self.pin_event = torch.cuda.Event()
        self.inflight = []              # (reader index, copy-done event) awaiting ring release
        self.rows = 0
        self.records = 0
        self.bytes = 0
        self.rejected = 0               # records whose header failed validation (dropped)

    def _dev_slot(self, nbytes: int) -> torch.Tensor:
        k = self.slot
        self.slot ^= 1
        buf = self.dev_buf[k]
        # the previous ingest that read this slot must be done before the copy overwrites it
        self.copy_stream.wait_event(self.dev_done[k])
        if buf.numel() < nbytes:
            torch.cuda.synchronize(self.rp.device)
            buf = torch.empty(int(nbytes * 1.25) + 4096, dtype=torch.uint8, device=self.rp.device)
            self.dev_buf[k] = buf
        return k

    def _release_done(self, wait: bool = False) -> None:
        keep = []
        for i, ev in self.inflight:
            if wait:
                ev.synchronize()
            if ev.query():
                self.readers[i].ring.release()
            else:
                keep.append((i, ev))
        self.inflight = keep

    def poll(self, max_records: int = 64) -> int:
        """Ingest up to ``max_records`` ready records (at most one per ring per call).  Returns the
        rows ingested."""
        self._release_done()
        busy = {i for i, _ in self.inflight}
        learner = self.stream if self.stream is not None else torch.cuda.current_stream(self.rp.device)
        rows_here, done = 0, 0
        big = False
        # dirty entries the poll's records may append before the single repair below: each kept
        # row can change one leaf; past half the list every later record skips it and the tree
        # is rebuilt (the kernel drops entries beyond max_dirty without a trace)
        budget, used = self.rp.max_dirty // 2, 0
        for i, r in enumerate(self.readers):
            if done >= max_records or i in busy:
                continue
            fr = r.ring.front()
            if fr is None:
                continue
            addr, n = fr
            n_rows = validate_record(np.frombuffer(ctypes.string_at(addr, min(n, header_bytes())),
                                                   np.uint8), n, self.rp.frame_bytes, 2 * self.rp.H)
            if n_rows is None:          # malformed: dropped before any DMA, never counted
                r.ring.release()
                self.rejected += 1
                continue
            k = self._dev_slot(n)
            dst = self.dev_buf[k]
            if self.registered[i] is not None:
                src = addr
            else:   # pinned bounce buffer: the previous DMA out of it must have finished
                if self.pinned is None or self.pinned.numel() < n:
                    self.pin_event.synchronize()
                    self.pinned = torch.empty(int(n * 1.25) + 4096, dtype=torch.uint8, pin_memory=True)
                self.pin_event.synchronize()
                ctypes.memmove(self.pinned.data_ptr(), addr, n)
                r.ring.release()
                src = self.pinned.data_ptr()
            check(kernels().r2_memcpy_h2d_async(_VP(ptr(dst)), _VP(src), n,
                                                _VP(self.copy_stream.cuda_stream)), "ingest h2d")
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            if self.registered[i] is not None:
                self.inflight.append((i, ev))
            else:
                self.pin_event.record(self.copy_stream)
            learner.wait_event(ev)
            kept = min(n_rows, self.rp.cap_e)
            use_dirty = not big and used + kept <= budget
            big |= not use_dirty
            used += kept if use_dirty else 0
            a = ingest_args(self.rp, ptr(dst), n, i, use_dirty)
            check(kernels().r2_ingest_record(ctypes.byref(a), _VP(stream_handle(learner))), "ingest")
            self.dev_done[k].record(learner)
            rows_here += min(n_rows, self.rp.cap_e)
            done += 1
            self.bytes += n
        if done:
            with torch.cuda.stream(learner):
                self.rp.repair_after_ingest(full=big)
            self.rows += rows_here
            self.records += done
            self.rp.total_written += rows_here
        return rows_here

    def check_errors(self) -> None:
        """Raise if the device ingest rejected a record (one D2H read; call at check points)."""
        if int(self.rp.ingest_err.item()) != 0:
            raise RuntimeError("device ingest rejected a malformed trajectory record")

    def close(self) -> None:
        self._release_done(wait=True)
        torch.cuda.synchronize(self.rp.device)
        for r, base in zip(self.readers, self.registered):
            if base is not None:
                kernels().r2_host_unregister(_VP(base))
            r.close()
