"""What bounds the fused split-precision GEMM (gemm_sp.hip)?  Times the engine's x-projection and
post-BPTT group GEMMs with the kernel's probe bits (r2_gemm5_set_mode bits 4-5):

  full      staging + LDS fragment reads + MFMAs (the production kernel)
  staging   operand DMA + waits + barriers only (no fragment reads, no MFMAs)
  compute   fragment reads + MFMAs on whatever the LDS holds (no DMA)

plus the same shapes as one bf16 product in hipBLASLt (torch.mm) and the library fp32 GEMM, as
attainable-rate reference points.

    python tools/gemm_sp_bound_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_r2d2_amd.ops._lib import kernels  # noqa: E402
from pytorch_r2d2_amd.ops.gemm import G5_CFGS, Gemm, gemm_sp, gemm_sp_ws_bytes  # noqa: E402

DEV = torch.device("cuda")


def split(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def timeit(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000.0


def main():
    k = kernels()
    g = torch.Generator(device=DEV).manual_seed(0)
    out = {}
    xs, xp = [], []
    for M in (5440, 5120):
        a = torch.randn(M, 1568, generator=g, device=DEV)
        w = torch.randn(1024, 1568, generator=g, device=DEV)
        xs.append((a, w))
        ah, al = split(a)
        bh, bl = split(w.t())
        xp.append(Gemm(ah, bh, torch.empty(M, 1024, device=DEV), bias=torch.randn(1024, device=DEV),
                       a_lo=al, b_lo=bl))
    probs = []
    for (M, N, K, ak) in [(1024, 1568, 2560, 0), (1024, 256, 2560, 0), (512, 256, 2560, 0),
                          (2560, 1568, 1024, 1)]:
        x = torch.randn(M, K, generator=g, device=DEV) if ak else \
            torch.randn(K, M, generator=g, device=DEV).t()
        y = torch.randn(K, N, generator=g, device=DEV).t().contiguous().t()
        xh, xl = split(x)
        yh, yl = split(y)
        if ak:
            ch = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            probs.append(Gemm(xh, yh, ch, a_lo=xl, b_lo=yl, c_lo=torch.empty_like(ch)))
        else:
            probs.append(Gemm(xh, yh, torch.zeros(M, N, device=DEV), a_lo=xl, b_lo=yl))
    splits = [4, 4, 4, 1]
    ws = torch.zeros(max(gemm_sp_ws_bytes(probs, splits, c) for c in range(len(G5_CFGS))) // 4 + 1,
                     device=DEV)
    tk = torch.zeros(4096, dtype=torch.int32, device=DEV)
    names = {0: "full", 1 << 4: "staging", 2 << 4: "compute"}
    for cfg in (-1, 3, 6):
        for bits, name in names.items():
            k.r2_gemm5_set_mode(1 | bits)
            out[f"xproj_cfg{cfg}_{name}_us"] = timeit(lambda: gemm_sp(xp, cfg=cfg))
            out[f"group_cfg{cfg}_{name}_us"] = timeit(
                lambda: gemm_sp(probs, splits=splits, cfg=cfg, ws=ws, tickets=tk))
    k.r2_gemm5_set_mode(1)
    # library reference points on the x-projection shapes (both nets, two calls)
    bf = [(a.to(torch.bfloat16), w.to(torch.bfloat16)) for a, w in xs]
    out["xproj_torch_bf16_us"] = timeit(lambda: [torch.mm(a, w.t()) for a, w in bf])
    out["xproj_torch_fp32_us"] = timeit(lambda: [torch.mm(a, w.t()) for a, w in xs])
    fl = sum(2.0 * a.shape[0] * 1024 * 1568 for a, _ in xs)
    out["xproj_gflop"] = fl / 1e9
    print(json.dumps({kk: round(v, 1) for kk, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
