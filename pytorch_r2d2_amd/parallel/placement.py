"""CU partitioning of one MI355X between co-located roles (actor group | learner).

An MI355X exposes 256 CUs in 8 XCDs.  A HIP stream can be restricted to a CU subset
(``hipExtStreamCreateWithCUMask``); measured on the device (``tools/cumask_probe.py``,
``profiles/archive/r02_cumask_probe.txt``): mask bit ``i`` selects a CU of XCD ``i % 8``, so the first
``8 k`` bits give every XCD ``k`` CUs and their complement gives every XCD ``32 - k``.  Both roles
therefore keep all 8 L2 slices and every XCD-aware tiling stays balanced.

The learner's persistent recurrence kernels need their whole grid co-resident at one workgroup
per CU; on a partitioned chip they are sized to the learner's CU count
(``LearnerEngine(n_cus=...)``), and the actor group -- whose kernels are all short, non-persistent
launches -- can never occupy the CUs those kernels wait for.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import torch

from ..ops._lib import kernels

N_XCD = 8


def cu_mask_words(n_cus: int, per_xcd: int, first: bool, n_xcd: int = N_XCD) -> List[int]:
    """32-bit mask words: ``first`` -> the ``per_xcd * n_xcd`` CUs of bits [0, per_xcd*n_xcd),
    else the complement (every remaining CU).  Every XCD must keep at least one CU in a mask: an
    XCD with none set runs the stream on ALL of its CUs (measured, tests/test_native_gpu.py
    partition test history: a mask of 8 CUs on XCDs 4-7 only ran on 32 CUs of XCDs 0-3 too)."""
    if n_cus % n_xcd or not 0 < per_xcd < n_cus // n_xcd:
        raise ValueError(f"cannot give {per_xcd} CUs per XCD out of {n_cus} CUs / {n_xcd} XCDs")
    cut = per_xcd * n_xcd
    bits = range(0, cut) if first else range(cut, n_cus)
    words = [0] * ((n_cus + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    return words


def xcd_counts(words: List[int], n_cus: int, n_xcd: int = N_XCD) -> List[int]:
    """CUs per XCD selected by a mask."""
    c = [0] * n_xcd
    for b in range(n_cus):
        if words[b // 32] >> (b % 32) & 1:
            c[b % n_xcd] += 1
    return c


class MaskedStream:
    """A HIP stream restricted to a CU mask, usable as a ``torch.cuda.Stream``."""

    def __init__(self, words: List[int], device=None):
        k = kernels()
        arr = (ctypes.c_uint32 * len(words))(*words)
        h = ctypes.c_void_p()
        rc = k.r2_stream_create_cumask(arr, len(words), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
        self.handle = h.value
        self.words = list(words)
        self.n_cus = sum(bin(w).count("1") for w in words)
        self.stream = torch.cuda.ExternalStream(self.handle, device=device)

    def mask(self) -> List[int]:
        got = (ctypes.c_uint32 * len(self.words))()
        kernels().r2_stream_get_cumask(ctypes.c_void_p(self.handle), got, len(self.words))
        return list(got)

    def close(self) -> None:
        if self.handle:
            torch.cuda.synchronize()
            kernels().r2_stream_destroy(ctypes.c_void_p(self.handle))
            self.handle = None


def split_chip(device, actor_cus_per_xcd: int = 4
               ) -> Tuple[Optional[MaskedStream], Optional[MaskedStream], int, int, Optional[List[int]]]:
    """(actor stream, learner stream, actor CUs, learner CUs, learner CUs per XCD).
    ``actor_cus_per_xcd`` <= 0: no partition (two ordinary streams sharing the chip; returns None
    streams): the learner keeps all 256 CUs for its placement and the actor's short kernels fill
    whatever CUs are idle at the moment -- safe because they never wait on the learner, so a
    persistent learner block that finds its CU taken only waits for an actor workgroup to end."""
    d = torch.device(device)
    n = int(torch.cuda.get_device_properties(d).multi_processor_count)
    if actor_cus_per_xcd <= 0:
        return None, None, n, n, None
    a = MaskedStream(cu_mask_words(n, actor_cus_per_xcd, True), d)
    lr = MaskedStream(cu_mask_words(n, actor_cus_per_xcd, False), d)
    return a, lr, a.n_cus, lr.n_cus, xcd_counts(lr.words, n)
