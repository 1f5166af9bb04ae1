"""Python bindings (ctypes) for the native host runtime ``_r2d2_runtime.so``.

See ``csrc/runtime/runtime.h``.  The library is built in-tree by ``pytorch_r2d2_amd._build``
(plain g++, no GPU needed) and is loaded lazily; it is independent of torch / HIP.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path
from typing import Optional, Tuple

import numpy as np

_SO = Path(__file__).resolve().parent.parent / "_r2d2_runtime.so"
_lib = None
_lock = threading.Lock()

P, I, I32, I64, U32, U64, D = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int32, ctypes.c_int64,
                               ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double)
_SIGS = {
    "r2rt_sumtree_create": (P, [I64]),
    "r2rt_sumtree_destroy": (None, [P]),
    "r2rt_sumtree_capacity": (I64, [P]),
    "r2rt_sumtree_set": (None, [P, P, P, I64]),
    "r2rt_sumtree_rebuild": (None, [P, P]),
    "r2rt_sumtree_total": (D, [P]),
    "r2rt_sumtree_get": (D, [P, I64]),
    "r2rt_sumtree_sample": (None, [P, P, I64, I, P, P]),
    "r2rt_ring_open": (P, [ctypes.c_char_p, U64, I]),
    "r2rt_ring_push": (I, [P, P, U32]),
    "r2rt_ring_pop": (I64, [P, P, U32]),
    "r2rt_ring_peek": (I64, [P]),
    "r2rt_ring_used": (U64, [P]),
    "r2rt_ring_front": (I64, [P, P]),
    "r2rt_ring_release": (None, [P]),
    "r2rt_ring_mapping": (P, [P, P]),
    "r2rt_slot_open": (P, [ctypes.c_char_p, U64, I]),
    "r2rt_slot_write": (None, [P, P, U64, I64]),
    "r2rt_slot_read": (I, [P, P, U64, I64, P]),
    "r2rt_slot_version": (I64, [P]),
    "r2rt_slot_close": (None, [P, I]),
    "r2rt_ring_capacity": (U64, [P]),
    "r2rt_ring_close": (None, [P, I]),
    "r2rt_lock_open": (I, [ctypes.c_char_p]),
    "r2rt_lock_acquire": (I, [I, I]),
    "r2rt_lock_release": (I, [I]),
    "r2rt_lock_close": (None, [I]),
    "r2rt_hb_open": (P, [ctypes.c_char_p, I, I]),
    "r2rt_hb_beat": (None, [P, I, U64, I32]),
    "r2rt_hb_read": (I, [P, I, P, P, P, P]),
    "r2rt_now_ns": (U64, []),
    "r2rt_hb_close": (None, [P, I]),
    "r2rt_version": (I, []),
}


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not _SO.exists():
                from .. import _build
                _build.build_runtime()
            l = ctypes.CDLL(str(_SO))
            for name, (res, args) in _SIGS.items():
                f = getattr(l, name)
                f.restype = res
                f.argtypes = args
            _lib = l
    return _lib


def now_ns() -> int:
    return int(lib().r2rt_now_ns())


class SumTree:
    """64-ary host sum tree (double precision) with batched updates and stratified sampling."""

    def __init__(self, capacity: int):
        self._h = lib().r2rt_sumtree_create(int(capacity))
        if not self._h:
            raise ValueError("bad capacity")
        self.capacity = int(capacity)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.r2rt_sumtree_destroy(h)
            self._h = None

    def set(self, idx, val) -> None:
        idx = np.ascontiguousarray(np.asarray(idx, dtype=np.int64).reshape(-1))
        val = np.ascontiguousarray(np.broadcast_to(np.asarray(val, dtype=np.float64), idx.shape))
        lib().r2rt_sumtree_set(self._h, idx.ctypes.data, val.ctypes.data, idx.size)

    def rebuild(self, leaves) -> None:
        leaves = np.ascontiguousarray(np.asarray(leaves, dtype=np.float64))
        assert leaves.size == self.capacity
        lib().r2rt_sumtree_rebuild(self._h, leaves.ctypes.data)

    def total(self) -> float:
        return float(lib().r2rt_sumtree_total(self._h))

    def get(self, idx: int) -> float:
        return float(lib().r2rt_sumtree_get(self._h, int(idx)))

    def sample(self, n: int, rng: Optional[np.random.Generator] = None,
               stratified: bool = True) -> Tuple[np.ndarray, np.ndarray]:
        rng = rng or np.random.default_rng()
        u = np.ascontiguousarray(rng.random(n))
        idx = np.empty(n, dtype=np.int64)
        p = np.empty(n, dtype=np.float64)
        lib().r2rt_sumtree_sample(self._h, u.ctypes.data, n, int(stratified), idx.ctypes.data,
                                  p.ctypes.data)
        return idx, p


class ShmRing:
    """SPSC byte ring in POSIX shared memory.  Exactly one producer and one consumer process."""

    def __init__(self, name: str, capacity: int, create: bool):
        self.name = name if name.startswith("/") else "/" + name
        self._h = lib().r2rt_ring_open(self.name.encode(), int(capacity), int(create))
        if not self._h:
            raise OSError(f"cannot open shm ring {self.name}")
        self.capacity = int(lib().r2rt_ring_capacity(self._h))
        self.owner = create
        self._buf = None

    def push(self, data) -> bool:
        """Returns False when the ring is full (caller retries / backs off)."""
        mv = memoryview(data).cast("B")
        buf = (ctypes.c_char * len(mv)).from_buffer_copy(mv) if mv.readonly else \
            (ctypes.c_char * len(mv)).from_buffer(mv)
        rc = lib().r2rt_ring_push(self._h, ctypes.addressof(buf), len(mv))
        if rc < 0:
            raise ValueError(f"record of {len(mv)} bytes exceeds ring capacity {self.capacity}")
        return rc == 0

    def pop(self) -> Optional[bytes]:
        n = lib().r2rt_ring_peek(self._h)
        if n < 0:
            return None
        if self._buf is None or len(self._buf) < n:
            self._buf = ctypes.create_string_buffer(max(int(n), 1 << 16))
        got = lib().r2rt_ring_pop(self._h, self._buf, len(self._buf))
        if got < 0:
            return None
        return self._buf.raw[:got]

    def front(self):
        """Zero-copy view of the front record: (address, length) or None.  The bytes stay valid
        (the producer cannot reuse them) until ``release()``."""
        p = ctypes.c_void_p()
        n = lib().r2rt_ring_front(self._h, ctypes.byref(p))
        if n < 0:
            return None
        return p.value, int(n)

    def release(self) -> None:
        lib().r2rt_ring_release(self._h)

    def mapping(self):
        """(address, bytes) of the whole shared mapping (for hipHostRegister)."""
        n = ctypes.c_uint64()
        base = lib().r2rt_ring_mapping(self._h, ctypes.byref(n))
        return int(base), int(n.value)

    def used(self) -> int:
        return int(lib().r2rt_ring_used(self._h))

    def close(self, unlink: Optional[bool] = None):
        if self._h:
            lib().r2rt_ring_close(self._h, int(self.owner if unlink is None else unlink))
            self._h = None

    def __del__(self):
        try:
            self.close(unlink=False)
        except Exception:
            pass


class ShmSlot:
    """Versioned blob in shared memory (seqlock): one writer process, any number of readers;
    a reader never observes a torn write."""

    def __init__(self, name: str, nbytes: int, create: bool):
        self.name = name if name.startswith("/") else "/" + name
        self.nbytes = int(nbytes)
        self._h = lib().r2rt_slot_open(self.name.encode(), self.nbytes, int(create))
        if not self._h:
            raise OSError(f"cannot open shm slot {self.name}")
        self.owner = create

    def write(self, arr: np.ndarray, version: int) -> None:
        a = np.ascontiguousarray(arr)
        if a.nbytes > self.nbytes:
            raise ValueError("blob larger than the slot")
        lib().r2rt_slot_write(self._h, a.ctypes.data, a.nbytes, int(version))

    def read(self, out: np.ndarray, have: int = -1) -> Optional[int]:
        """Copy a version newer than ``have`` into ``out``; returns its version or None."""
        v = ctypes.c_int64()
        rc = lib().r2rt_slot_read(self._h, out.ctypes.data, out.nbytes, int(have), ctypes.byref(v))
        return int(v.value) if rc == 1 else None

    def version(self) -> int:
        return int(lib().r2rt_slot_version(self._h))

    def close(self, unlink: Optional[bool] = None):
        if self._h:
            lib().r2rt_slot_close(self._h, int(self.owner if unlink is None else unlink))
            self._h = None

    def __del__(self):
        try:
            self.close(unlink=False)
        except Exception:
            pass


class FileLock:
    """fcntl write lock on ``path + '.lock'`` (never the data file itself)."""

    def __init__(self, path: str):
        self.path = path + ".lock"
        os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        self.fd = lib().r2rt_lock_open(self.path.encode())
        if self.fd < 0:
            raise OSError(f"cannot open lock {self.path}")
        self.held = False

    def acquire(self, blocking: bool = True) -> bool:
        rc = lib().r2rt_lock_acquire(self.fd, int(blocking))
        if rc < 0:
            raise OSError("fcntl lock failed")
        self.held = rc == 1
        return self.held

    def release(self) -> None:
        if self.held:
            lib().r2rt_lock_release(self.fd)
            self.held = False

    def close(self):
        if self.fd >= 0:
            self.release()
            lib().r2rt_lock_close(self.fd)
            self.fd = -1

    def __enter__(self):
        self.acquire(True)
        return self

    def __exit__(self, *a):
        self.release()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HeartbeatTable:
    def __init__(self, name: str, n_slots: int, create: bool):
        self.name = name if name.startswith("/") else "/" + name
        self.n = n_slots
        self._h = lib().r2rt_hb_open(self.name.encode(), int(n_slots), int(create))
        if not self._h:
            raise OSError(f"cannot open heartbeat table {self.name}")
        self.owner = create

    def beat(self, slot: int, counter: int = 0, status: int = 0) -> None:
        lib().r2rt_hb_beat(self._h, slot, int(counter), int(status))

    def read(self, slot: int):
        last, cnt = ctypes.c_uint64(), ctypes.c_uint64()
        pid, st = ctypes.c_int32(), ctypes.c_int32()
        lib().r2rt_hb_read(self._h, slot, ctypes.byref(last), ctypes.byref(cnt), ctypes.byref(pid),
                           ctypes.byref(st))
        return {"last_ns": last.value, "counter": cnt.value, "pid": pid.value, "status": st.value}

    def age_s(self, slot: int) -> float:
        r = self.read(slot)
        if r["last_ns"] == 0:
            return float("inf")
        return (now_ns() - r["last_ns"]) / 1e9

    def close(self, unlink: Optional[bool] = None):
        if self._h:
            lib().r2rt_hb_close(self._h, int(self.owner if unlink is None else unlink))
            self._h = None


__all__ = ["SumTree", "ShmRing", "ShmSlot", "FileLock", "HeartbeatTable", "now_ns", "lib"]
