"""Python front end of the batched MFMA GEMM (csrc/kernels/gemm.hip).

A problem computes  C (=|+=) alpha * A @ B (+ bias)  with bf16 operands given as strided 2-D
views; each operand may be K-contiguous or M/N-contiguous (the kernel stages the latter with
hardware-transposed LDS reads), so transposed products such as ``dz.t() @ h`` need no copies.
Output fp32 or bf16, optional per-column bias and an output row map (``crow[m]`` = row of C
that receives row m of the product)."""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from ._lib import check, kernels, stream_handle


def _layout(x: torch.Tensor, rows_are_outer: bool):
    """Classify a 2-D view X[i][k] (i = outer M/N index, k = reduction index).
    Returns (kmajor, ld)."""
    si, sk = x.stride()
    if sk == 1:
        return 1, si
    if si == 1:
        return 0, sk
    raise ValueError("gemm operand must be contiguous in one dimension")


@dataclass
class Gemm:
    a: torch.Tensor          # (M, K) view
    b: torch.Tensor          # (K, N) view
    c: torch.Tensor          # (M_out, N) fp32 or bf16, row stride ldc, unit column stride
    bias: Optional[torch.Tensor] = None
    crow: Optional[torch.Tensor] = None
    accumulate: bool = False
    alpha: float = 1.0
    # split precision (csrc/split.h): lo planes with the same shape / strides as a, b, c
    a_lo: Optional[torch.Tensor] = None
    b_lo: Optional[torch.Tensor] = None
    c_lo: Optional[torch.Tensor] = None

    def desc(self) -> List[int]:
        a, b, c = self.a, self.b, self.c
        for x, lo in ((a, self.a_lo), (b, self.b_lo), (c, self.c_lo)):
            if lo is not None:
                assert lo.shape == x.shape and lo.stride() == x.stride() and lo.dtype == torch.bfloat16
        assert a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
        M, K = a.shape
        K2, N = b.shape
        assert K == K2, (a.shape, b.shape)
        ak, lda = _layout(a, True)                 # A[m][k]
        bk, ldb = _layout(b.t(), True)             # B^T[n][k]
        assert c.stride(1) == 1 and c.dtype in (torch.float32, torch.bfloat16)
        if self.crow is None:
            assert c.shape[0] >= M and c.shape[1] >= N
        alpha_bits = struct.unpack("<I", struct.pack("<f", float(self.alpha)))[0]
        return [a.data_ptr(), b.data_ptr(), c.data_ptr(),
                0 if self.bias is None else self.bias.data_ptr(),
                0 if self.crow is None else self.crow.data_ptr(),
                M, N, K, lda, ldb, c.stride(0), ak, bk, int(c.dtype == torch.float32),
                int(self.accumulate), alpha_bits,
                0 if self.a_lo is None else self.a_lo.data_ptr(),
                0 if self.b_lo is None else self.b_lo.data_ptr(),
                0 if self.c_lo is None else self.c_lo.data_ptr(), 0]


def gemm(*problems: Gemm, stream=None) -> None:
    """Run up to 4 problems sharing one operand-layout combination in one launch."""
    arr = np.asarray([v for p in problems for v in p.desc()], dtype=np.int64)
    check(kernels().r2_gemm(arr.ctypes.data, len(problems), stream or stream_handle()), "gemm")


def group_ws_bytes(problems: List[Gemm], splits: List[int]) -> int:
    """Workspace of :func:`gemm_group` (64 KB fp32 partial per split item)."""
    total = 0
    for p, sp in zip(problems, splits):
        M, N = p.a.shape[0], p.b.shape[1]
        if sp > 1:
            total += ((M + 127) // 128) * ((N + 127) // 128) * sp * 65536
    return total


def gemm_group(problems: List[Gemm], splits: List[int], ws: torch.Tensor, tickets: torch.Tensor,
               stream=None) -> None:
    """Up to 4 problems (any A layout, mn-major B, K % 64 == 0) in ONE launch, problem i's K
    split ``splits[i]`` ways with a deterministic last-arriver reduction (gemm.hip
    gemm_group_kernel).  ``tickets`` int32 zeros, >= total tiles of the split problems."""
    arr = np.asarray([v for p in problems for v in p.desc()], dtype=np.int64)
    sp = np.asarray(splits, dtype=np.int32)
    check(kernels().r2_gemm_group(arr.ctypes.data, sp.ctypes.data, len(problems), ws.data_ptr(),
                                  ws.numel() * ws.element_size(), tickets.data_ptr(), tickets.numel(),
                                  stream or stream_handle()), "gemm_group")


_G5_WS = {}
# csrc/kernels/gemm_sp.hip g5_cfgs: (BM, BN, BK, stages)
G5_CFGS = [(192, 128, 64, 2), (128, 128, 64, 2), (256, 128, 32, 3), (256, 256, 32, 2),
           (256, 64, 64, 2), (128, 64, 64, 2), (128, 128, 32, 4), (192, 256, 32, 2)]


def gemm_sp(problems: List[Gemm], splits: Optional[List[int]] = None, cfg: int = -1,
            ws: Optional[torch.Tensor] = None, tickets: Optional[torch.Tensor] = None,
            n_cus: int = 0, stream=None) -> int:
    """Fused split-precision GEMM (csrc/kernels/gemm_sp.hip): up to 4 problems (every operand
    split, shared B layout, any A layout) in one launch, each with a K split; all three hi / lo
    products from ONE pass over K.  ``splits``: K split per problem, 0 = automatic (spread a
    small-M problem's K over CUs the launch leaves idle, gemm_sp.hip g5_auto_split).  ``cfg``:
    index into ``G5_CFGS`` or -1 = the launcher picks the tile for ``n_cus`` CUs.  ``ws`` /
    ``tickets``: split-K workspace (fp32) and zeroed int32
    tickets; allocated (and cached per device) when omitted -- pass them explicitly inside a graph
    capture.  Returns the configuration used."""
    arr = np.asarray([v for p in problems for v in p.desc()], dtype=np.int64)
    sp = np.asarray(splits if splits is not None else [1] * len(problems), dtype=np.int32)
    k = kernels()
    if ws is None or tickets is None:
        dev = problems[0].c.device
        need = 0
        if (sp != 1).any():
            for c in ([cfg] if cfg >= 0 else range(len(G5_CFGS))):
                need = max(need, int(k.r2_gemm5_ws_bytes_nc(arr.ctypes.data, sp.ctypes.data,
                                                            len(problems), c, int(n_cus))))
        key = str(dev)
        cur = _G5_WS.get(key)
        if cur is None or cur[0].numel() * 4 < need:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("gemm_sp: pass ws / tickets when capturing a graph")
            cur = (torch.zeros(max(need // 4, 1), dtype=torch.float32, device=dev),
                   torch.zeros(4096, dtype=torch.int32, device=dev))
            _G5_WS[key] = cur
        ws, tickets = cur
    rc = k.r2_gemm5(arr.ctypes.data, sp.ctypes.data, len(problems), int(cfg), ws.data_ptr(),
                    ws.numel() * ws.element_size(), tickets.data_ptr(), tickets.numel(), int(n_cus),
                    stream or stream_handle())
    if rc < 0:
        raise RuntimeError(f"gemm_sp failed with code {rc}")
    return rc


def gemm_sp_ws_bytes(problems: List[Gemm], splits: List[int], cfg: int, n_cus: int = 0) -> int:
    arr = np.asarray([v for p in problems for v in p.desc()], dtype=np.int64)
    sp = np.asarray(splits, dtype=np.int32)
    return int(kernels().r2_gemm5_ws_bytes_nc(arr.ctypes.data, sp.ctypes.data, len(problems), cfg,
                                              int(n_cus)))
