"""Split GEMMs of the fp32 step on gemm5 vs gemm6 (fragment registers refilled between the three
product passes): the x-projection of both nets (5440 / 5120 x 1568 . 1568 x 1024, fp32 out +
bias) and the post-BPTT group (dW_ih, dW_hh, dW_head1 with mn-major A, dX with split output; K
splits 4,4,4,1), time and error vs float64.

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
    probs, grefs = [], []
    for (M, N, K, ak) in [(1024, 1568, 2560, 0), (1024, 256, 2560, 0), (512, 256, 2560, 0),
                          (2560, 1568, 1024, 1)]:
        x = torch.randn(M, K, generator=g, device=DEV) if ak else \
            torch.randn(K, M, generator=g, device=DEV).t()
        y = torch.randn(N, K, generator=g, device=DEV).t().contiguous()
        xh, xl = split(x)
        yh, yl = split(y)
        if ak:
            ch = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            probs.append(Gemm(xh, yh, ch, a_lo=xl, b_lo=yl, c_lo=torch.empty_like(ch)))
        else:
            probs.append(Gemm(xh, yh, torch.zeros(M, N, device=DEV), a_lo=xl, b_lo=yl))
        grefs.append(x.double() @ y.double())
    splits = [4, 4, 4, 1]

    def group():
        for p in probs[:3]:
            p.c.zero_()
        return gemm_sp(probs, splits=splits)

    def gerr():
        e = 0.0
        for p, r in zip(probs, grefs):
            c = p.c.double() + (p.c_lo.double() if p.c_lo is not None else 0)
            e = max(e, ((c - r).norm() / r.norm()).item())
        return e
    for name, mode in (("gemm5", 1 | 4), ("gemm6", 1), ("gemm5_again", 1 | 4), ("gemm6_again", 1)):
        k.r2_gemm5_set_mode(mode)
        for p in xp:
            p.c.zero_()
        cfg = gemm_sp(xp, cfg=7)
        torch.cuda.synchronize()
        err = max(((p.c.double() - r).norm() / r.norm()).item() for p, r in zip(xp, refs))
        out[name + "_us"] = timeit(lambda: gemm_sp(xp, cfg=7))
        out[name + "_relerr"] = err
        out[name + "_cfg"] = cfg
        out[name + "_group_cfg"] = group()
        torch.cuda.synchronize()
        out[name + "_group_relerr"] = gerr()
        out[name + "_group_us"] = timeit(group)
    k.r2_gemm5_set_mode(1)
    flops = 2 * 3 * (5440 + 5120) * 1024 * 1568
    out["gemm6_tflops_3pass"] = round(flops / out["gemm6_us"] / 1e6, 1)
    out["gemm5_tflops_3pass"] = round(flops / out["gemm5_us"] / 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
