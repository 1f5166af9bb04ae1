"""x-projection split GEMM (both nets, atari57: 5440 / 5120 x 1568 . 1568 x 1024, fp32 out + bias):
gemm5 (8 waves, 192 x 256) vs gemm6 (4 waves, 1 per SIMD, fragment refill between passes), time
and error vs float64.

    python tools/gemm6_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_r2d2_amd.ops._lib import kernels  # noqa: E402
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm_sp  # noqa: E402

DEV = torch.device("cuda")


def split(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1000.0, 1)


def main():
    g = torch.Generator(device=DEV).manual_seed(0)
    xp, refs = [], []
    for M in (5440, 5120):
        a = torch.randn(M, 1568, generator=g, device=DEV)
        w = torch.randn(1024, 1568, generator=g, device=DEV)
        bias = torch.randn(1024, generator=g, device=DEV)
        ah, al = split(a)
        wh, wl = split(w)
        xp.append(Gemm(ah, wh.t(), torch.empty(M, 1024, device=DEV), bias=bias, a_lo=al, b_lo=wl.t()))
        refs.append((a.double() @ w.double().t() + bias.double()))
    k = kernels()
    out = {}
    for name, mode in (("gemm5", 1 | 4), ("gemm6", 1), ("gemm6_nw4", 1 | 8), ("gemm5_again", 1 | 4), ("gemm6_again", 1)):
        k.r2_gemm5_set_mode(mode)
        for p in xp:
            p.c.zero_()
        cfg = gemm_sp(xp, cfg=7)
        torch.cuda.synchronize()
        err = max(((p.c.double() - r).norm() / r.norm()).item() for p, r in zip(xp, refs))
        out[name + "_us"] = timeit(lambda: gemm_sp(xp, cfg=7))
        out[name + "_relerr"] = err
        out[name + "_cfg"] = cfg
    k.r2_gemm5_set_mode(1)
    flops = 2 * 3 * (5440 + 5120) * 1024 * 1568
    out["gemm6_tflops_3pass"] = round(flops / out["gemm6_us"] / 1e6, 1)
    out["gemm5_tflops_3pass"] = round(flops / out["gemm5_us"] / 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
