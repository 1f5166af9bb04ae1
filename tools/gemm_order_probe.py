"""Item order of the K-split split GEMMs (gemm_sp.hip g5_coords, r2_gemm5_set_mode bit 6) on the
post-BPTT group of the paper config (dW_ih 1024 x 1568, dW_hh 1024 x 256, dW_head1 512 x 256 with
K = 2560 and mn-major A; dX 2560 x 1568 x 1024 with hi / lo output), splits 3,3,3,1 on the
128 x 128 4-deep tile (the engine's choice): rounds of the two orders interleaved in one process,
us per launch, and whether the outputs are bitwise equal (the split-K reduction sums the slabs in
K order either way).

    python tools/gemm_order_probe.py
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


def timeit(fn, n=40):
    for _ in range(3):
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
    probs = []
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
    k = kernels()
    out = {"rounds": []}
    results = {}
    for splits, cfg in (([3, 3, 3, 1], 6), ([4, 4, 4, 1], 6)):
        key = f"splits{''.join(map(str, splits))}_cfg{cfg}"
        for rnd in range(4):
            row = {"case": key, "round": rnd}
            for order in (0, 1):
                k.r2_gemm5_set_mode(1 | (0 if order else 64))   # bit 6: tile-major order

                def run():
                    for p in probs[:3]:
                        p.c.zero_()
                    gemm_sp(probs, splits=splits, cfg=cfg)
                row[f"order{order}_us"] = timeit(run)
                run()
                torch.cuda.synchronize()
                results[order] = [p.c.clone() for p in probs] + [probs[3].c_lo.clone()]
            row["bitwise_equal"] = all(torch.equal(a, b) for a, b in zip(results[0], results[1]))
            out["rounds"].append(row)
            print(json.dumps(row), flush=True)
    k.r2_gemm5_set_mode(1)


if __name__ == "__main__":
    main()
