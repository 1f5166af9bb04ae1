"""Tile configurations of the split-precision heads layer-1 GEMM (three heads in one gemm_sp
launch: z = h . W1^T, M 3 x 2560, N 512, K 256, fp32 out) -- time per config and the
launcher's own pick (cfg -1), error vs float64.

    python tools/heads_gemm_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_r2d2_amd.ops.gemm import G5_CFGS, Gemm, gemm_sp  # noqa: E402

DEV = torch.device("cuda")


def split(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def timeit(fn, n=20):
    """Kernel time per launch: n launches captured in one HIP graph (host-side argument packing
    stays out of the timed replay)."""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / (5 * n) * 1000.0, 1)


def main():
    g = torch.Generator(device=DEV).manual_seed(0)
    probs, refs = [], []
    for M in (2560, 2560, 2560):
        h = torch.randn(M, 256, generator=g, device=DEV)
        w = torch.randn(512, 256, generator=g, device=DEV) * 0.05
        hh, hl = split(h)
        wh, wl = split(w)
        probs.append(Gemm(hh, wh.t(), torch.empty(M, 512, device=DEV), a_lo=hl, b_lo=wl.t()))
        refs.append(h.double() @ w.double().t())
    out = {"auto_cfg": gemm_sp(probs, cfg=-1, n_cus=256)}
    out["auto_us"] = timeit(lambda: gemm_sp(probs, cfg=-1, n_cus=256))
    for c in range(len(G5_CFGS)):
        try:
            gemm_sp(probs, cfg=c)
        except RuntimeError as e:
            out[f"cfg{c}"] = str(e)
            continue
        torch.cuda.synchronize()
        err = max(((p.c.double() - r).norm() / r.norm()).item() for p, r in zip(probs, refs))
        out[f"cfg{c}_{G5_CFGS[c][0]}x{G5_CFGS[c][1]}"] = [timeit(lambda: gemm_sp(probs, cfg=c)), f"{err:.1e}"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
