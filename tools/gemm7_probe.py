"""x-projection of the fp32 step (both nets: 5440 / 5120 x 1568 . 1568 x 1024, fp32 out + bias,
every operand split) on gemm6 vs gemm7 (gemm_sp.hip: deep LDS-DMA ring of 16-deep K tiles),
192 x 256 and 256 x 256 tiles, interleaved rounds in one process; error vs float64 and the max
abs difference between the two kernels' outputs.

    python tools/gemm7_probe.py [rounds]
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    g = torch.Generator(device=DEV).manual_seed(0)
    xp, refs = [], []
    for M in (5440, 5120):
        a = torch.relu(torch.randn(M, 1568, generator=g, device=DEV))
        w = torch.randn(1024, 1568, generator=g, device=DEV) * 0.02
        bias = torch.randn(1024, generator=g, device=DEV)
        ah, al = split(a)
        wh, wl = split(w)
        xp.append(Gemm(ah, wh.t(), torch.empty(M, 1024, device=DEV), bias=bias, a_lo=al, b_lo=wl.t()))
        refs.append(a.double() @ w.double().t() + bias.double())
    # post-BPTT group: dW_ih, dW_hh, dW_head1 (mn-major A), dX (k-major A, split output); B mn-major
    probs, grefs = [], []
    for (M, N, K, ak) in [(1024, 1568, 2560, 0), (1024, 256, 2560, 0), (512, 256, 2560, 0),
                          (2560, 1568, 1024, 1)]:
        x = torch.randn(M, K, generator=g, device=DEV) if ak else \
            torch.randn(K, M, generator=g, device=DEV).t()
        y = torch.randn(K, N, generator=g, device=DEV)
        xh, xl = split(x)
        yh, yl = split(y)
        if ak:
            ch = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            probs.append(Gemm(xh, yh, ch, a_lo=xl, b_lo=yl, c_lo=torch.empty_like(ch)))
        else:
            probs.append(Gemm(xh, yh, torch.zeros(M, N, device=DEV), a_lo=xl, b_lo=yl))
        grefs.append(x.double() @ y.double())

    def group():
        for p in probs[:3]:
            p.c.zero_()
        return gemm_sp(probs, splits=[4, 4, 4, 1], cfg=3)

    def gerr():
        e = 0.0
        for p, r in zip(probs, grefs):
            c = p.c.double() + (p.c_lo.double() if p.c_lo is not None else 0)
            e = max(e, ((c - r).norm() / r.norm()).item())
        return e
    k = kernels()
    out = {}
    outs = {}
    for name, mode in (("group_g6", 1), ("group_g7", 1 | 8)):
        k.r2_gemm5_set_mode(mode)
        group()
        torch.cuda.synchronize()
        out[name + "_relerr"] = gerr()
    arms = (("g6_192", 1, 7), ("g7_192", 1 | 8, 7), ("g6_256", 1, 3), ("g7_256", 1 | 8, 3))
    for name, mode, cfg in arms:
        k.r2_gemm5_set_mode(mode)
        for p in xp:
            p.c.fill_(float("nan"))
        gemm_sp(xp, cfg=cfg)
        torch.cuda.synchronize()
        out[name + "_relerr"] = max(((p.c.double() - r).norm() / r.norm()).item()
                                    for p, r in zip(xp, refs))
        outs[name] = [p.c.clone() for p in xp]
    for a_, b_ in (("g6_192", "g7_192"), ("g6_256", "g7_256")):
        out[f"maxdiff_{a_}_{b_}"] = max((x - y).abs().max().item() for x, y in zip(outs[a_], outs[b_]))
    for r in range(rounds):
        for name, mode, cfg in arms:
            k.r2_gemm5_set_mode(mode)
            out.setdefault(name + "_us", []).append(timeit(lambda: gemm_sp(xp, cfg=cfg)))
        for name, mode in (("group_g6", 1), ("group_g7", 1 | 8)):
            k.r2_gemm5_set_mode(mode)
            out.setdefault(name + "_us", []).append(timeit(group))
    # probe arms (mode bits 4-5 = G5Args::dbg): 1 = operand staging only, 2 = no staging
    # (gemm5 for the 2-stage 32-deep structure, gemm7 for the deep ring)
    if len(sys.argv) > 2:
        for name, mode in (("g5_192", 1 | 4), ("g5_192_stage_only", 1 | 4 | 16),
                           ("g5_192_no_stage", 1 | 4 | 32), ("g7_192_stage_only", 1 | 8 | 16),
                           ("g7_192_no_stage", 1 | 8 | 32)):
            k.r2_gemm5_set_mode(mode)
            out[name + "_us"] = timeit(lambda: gemm_sp(xp, cfg=7))
    k.r2_gemm5_set_mode(1)
    flops = 2 * 3 * (5440 + 5120) * 1024 * 1568
    for name, _, _ in arms:
        out[name + "_tflops_3pass"] = round(flops / min(out[name + "_us"]) / 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
