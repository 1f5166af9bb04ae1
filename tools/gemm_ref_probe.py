"""Reference ceiling for the split GEMMs of the fp32 step: hipBLASLt (torch.mm, bf16 operands,
fp32 output) on the same shapes and random data as the hand-written split kernel
(gemm_sp.hip), one pass and the three hi / lo passes, beside gemm_sp itself.

    python tools/gemm_ref_probe.py            # one JSON line (microseconds per call)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_r2d2_amd.ops.gemm import Gemm, gemm_sp  # noqa: E402

DEV = torch.device("cuda")


def split(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def timeit(fn, n=40):
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
    out = {}
    # x-projection of both nets: (5440 | 5120) x 1568 . 1568 x 1024
    xs = [torch.randn(M, 1568, device=DEV, generator=g) for M in (5440, 5120)]
    ws = [torch.randn(1024, 1568, device=DEV, generator=g) * 0.03 for _ in range(2)]
    xsp = [split(x) for x in xs]
    wsp = [split(w) for w in ws]
    cs = [torch.empty(x.shape[0], 1024, device=DEV) for x in xs]

    def blas1():
        for (xh, _), (wh, _), c in zip(xsp, wsp, cs):
            torch.mm(xh, wh.t(), out_dtype=torch.float32, out=c)

    def blas3():
        for (xh, xl), (wh, wl), c in zip(xsp, wsp, cs):
            torch.mm(xh, wh.t(), out_dtype=torch.float32, out=c)
            c.add_(torch.mm(xh, wl.t(), out_dtype=torch.float32))
            c.add_(torch.mm(xl, wh.t(), out_dtype=torch.float32))

    out["xproj_blaslt_1pass_us"] = timeit(blas1)
    out["xproj_blaslt_3pass_us"] = timeit(blas3)
    probs = [Gemm(xh, wh.t(), c, a_lo=xl, b_lo=wl.t()) for (xh, xl), (wh, wl), c in zip(xsp, wsp, cs)]
    out["xproj_gemm_sp_us"] = timeit(lambda: gemm_sp(probs))
    flop = 2 * 10560 * 1024 * 1568
    out["xproj_blaslt_1pass_tflops"] = round(flop / out["xproj_blaslt_1pass_us"] / 1e6, 1)
    out["xproj_gemm_sp_tflops_3x"] = round(3 * flop / out["xproj_gemm_sp_us"] / 1e6, 1)
    # one big square-ish bf16 GEMM for the chip's library ceiling on random data
    a = torch.randn(8192, 8192, device=DEV, generator=g).to(torch.bfloat16)
    b = torch.randn(8192, 8192, device=DEV, generator=g).to(torch.bfloat16)
    t = timeit(lambda: torch.mm(a, b), n=10)
    out["blaslt_8192cube_tflops"] = round(2 * 8192 ** 3 / t / 1e6, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
