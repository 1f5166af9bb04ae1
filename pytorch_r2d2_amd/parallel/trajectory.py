"""Actor -> learner trajectory push.

Reference: actors pickle their whole 50k-row replay to ``./logs/memory/memory{id}.pt`` every 5
episodes under a fasteners lock; the learner polls, unpickles, extends its ring and deletes the
file (replay_memory.py:125-173) -- 233 MB per 5k rows, 1.5 s save / 1.2 s load.

Two MI355X-native transports, both moving *packed rows* (uint8 frames + fp32 [h|c] x2 +
scalars, the §2.5 schema) in fixed-size chunks:

* ``parallel/channel.py`` + ``parallel/actor_ranks.py`` -- GPU actor groups on one rank, learner
  replay shard on another: records packed on the device, sent over asynchronous RCCL links,
  received into device memory and scattered into the HBM replay by the ingest kernel -- the
  bytes never visit the host.
* ``ShmTrajectoryWriter/Reader`` -- CPU actor processes on the same host: records go through
  the native shared-memory SPSC ring (``runtime.ShmRing``) -- no files, no pickles, no locks --
  and the learner DMAs them into HBM (``engine/ingest.py``).

``pack_rows`` / ``unpack_rows`` define the wire format (a single uint8 buffer: header + SoA
fields at 64-byte aligned offsets, ``record_layout``).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..runtime import ShmRing

ORDER = ("state", "hs_cs", "target_hs_cs", "action", "reward", "done", "stack_count",
         "priority", "sequence_priority", "is_seq_start")
MAGIC = 0x52324454  # "R2DT"


ALIGN = 64          # every field starts 64-byte aligned (16-byte vector loads on the device)
CODES = {np.dtype(np.uint8): 0, np.dtype(np.int8): 1, np.dtype(np.float32): 2}


def _pad(x: int) -> int:
    return (x + ALIGN - 1) // ALIGN * ALIGN


def record_layout(buf_head: np.ndarray):
    """Parse a record header -> (n_rows, {name: (code, per_row, nbytes, byte offset)})."""
    head = np.asarray(buf_head[:24], dtype=np.uint8).view(np.int64)
    if int(head[0]) != MAGIC:
        raise ValueError("bad trajectory record")
    n, k = int(head[1]), int(head[2])
    meta = np.asarray(buf_head[24:24 + 24 * k], dtype=np.uint8).view(np.int64).reshape(k, 3)
    off = _pad(24 + 24 * k)
    fields = {}
    for name, (code, per_row, nbytes) in zip(ORDER, meta):
        fields[name] = (int(code), int(per_row), int(nbytes), off)
        off += _pad(int(nbytes))
    return n, fields


def validate_record(buf_head: np.ndarray, rec_bytes: int, frame_bytes: int, h2: int):
    """Host mirror of ``parse_record`` (csrc/kernels/ingest.hip): the row count of a record whose
    header matches the replay schema and whose fields hold all of their rows, else None."""
    try:
        head = np.asarray(buf_head[:24], dtype=np.uint8).view(np.int64)
        if int(head[0]) != MAGIC or int(head[2]) != len(ORDER):
            return None
        n, fields = record_layout(buf_head)
    except ValueError:
        return None
    end = max(off + _pad(nb) for _, _, nb, off in fields.values())
    if n < 0 or end > rec_bytes:
        return None
    for code, per_row, nbytes, _ in fields.values():
        if code not in (0, 1, 2) or per_row < 1 or nbytes < n * per_row * (4 if code == 2 else 1):
            return None
    c = {k: v[:2] for k, v in fields.items()}
    if c["state"] != (0, frame_bytes) or c["hs_cs"] != (2, h2) or c["target_hs_cs"] != (2, h2):
        return None
    if any(c[k][0] != 2 for k in ("reward", "priority", "sequence_priority")):
        return None
    if c["action"][0] == 2 or c["is_seq_start"][0] == 2:
        return None
    return n


def record_spec(n_rows: int, frame_bytes: int, h2: int):
    """The record layout ``pack_rows`` produces for ``n_rows`` rows of the replay schema (uint8
    frames, fp32 [h|c] x 2, int8 action / stack count, fp32 reward / done / priorities, uint8
    start flag) without
    materialising the rows: (header uint8 array, byte offset of every field, total bytes).  The
    device pack kernel (csrc/kernels/ingest.hip pack_rows_kernel) fills the fields of a buffer
    whose header was written once from this."""
    # the reference's dtypes (replay_memory.py:76-87): action int8, done fp32
    spec = [(0, frame_bytes, 1), (2, h2, 4), (2, h2, 4), (1, 1, 1), (2, 1, 4), (2, 1, 4), (1, 1, 1),
            (2, 1, 4), (2, 1, 4), (0, 1, 1)]
    meta, offs = [], []
    off = header_bytes()
    for code, per_row, esz in spec:
        nb = n_rows * per_row * esz
        meta += [code, per_row, nb]
        offs.append(off)
        off += _pad(nb)
    hdr = np.zeros(header_bytes(), dtype=np.uint8)
    h = np.asarray([MAGIC, n_rows, len(ORDER)] + meta, dtype=np.int64).view(np.uint8)
    hdr[: h.size] = h
    return hdr, offs, off


def header_bytes(k: int = len(ORDER)) -> int:
    return _pad(24 + 24 * k)


def pack_rows(mem: Dict[str, np.ndarray]) -> np.ndarray:
    """Row-schema dict -> one contiguous uint8 record: header int64 x (3 + 3*K), then every field
    (SoA, the §2.5 schema) at a 64-byte aligned offset."""
    n = int(np.asarray(mem["state"]).shape[0])
    arrs, meta = [], []
    for k in ORDER:
        a = np.ascontiguousarray(np.asarray(mem[k]))
        if a.dtype == np.bool_:
            a = a.astype(np.uint8)
        per_row = int(a.size // max(n, 1)) if n else int(np.prod(a.shape[1:]))
        meta += [CODES[a.dtype], per_row, a.nbytes]
        arrs.append(a)
    total = header_bytes() + sum(_pad(a.nbytes) for a in arrs)
    out = np.zeros(total, dtype=np.uint8)
    hdr = np.asarray([MAGIC, n, len(ORDER)] + meta, dtype=np.int64).view(np.uint8)
    out[: hdr.size] = hdr
    off = header_bytes()
    for a in arrs:
        out[off: off + a.nbytes] = a.view(np.uint8).reshape(-1)
        off += _pad(a.nbytes)
    return out


def unpack_rows(buf: np.ndarray, state_shape=None) -> Dict[str, np.ndarray]:
    buf = np.asarray(buf, dtype=np.uint8)
    n, fields = record_layout(buf)
    out = {}
    dts = {0: np.uint8, 1: np.int8, 2: np.float32}
    for name, (code, per_row, nbytes, off) in fields.items():
        a = buf[off:off + nbytes].view(dts[code])
        if name == "state" and state_shape is not None:
            a = a.reshape(n, *state_shape)
        elif per_row > 1:
            a = a.reshape(n, per_row)
        elif name in ("action", "reward", "done"):
            a = a.reshape(n, 1)
        out[name] = a
    return out


class ShmTrajectoryWriter:
    def __init__(self, name: str, capacity: int = 256 << 20):
        self.ring = ShmRing(name, capacity, create=False)
        self.dropped = 0

    def push(self, mem: Dict[str, np.ndarray], block: bool = True, spin_s: float = 0.001) -> bool:
        import time
        rec = pack_rows(mem)
        while not self.ring.push(rec):
            if not block:
                self.dropped += 1
                return False
            time.sleep(spin_s)
        return True


class ShmTrajectoryReader:
    def __init__(self, name: str, capacity: int = 256 << 20, state_shape=None):
        self.ring = ShmRing(name, capacity, create=True)
        self.state_shape = state_shape

    def poll(self, max_records: int = 64) -> List[Dict[str, np.ndarray]]:
        out = []
        for _ in range(max_records):
            rec = self.ring.pop()
            if rec is None:
                break
            out.append(unpack_rows(np.frombuffer(rec, dtype=np.uint8), self.state_shape))
        return out

    def close(self):
        self.ring.close(unlink=True)
