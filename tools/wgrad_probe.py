"""The post-BPTT weight-gradient GEMMs of the fp32 paper step (dW_ih 1024x1568, dW_hh 1024x256,
dW_head1 512x256, K = 2560 time-major rows; every operand split, mn-major A and B) on the fused
split GEMM (gemm_sp.hip), per tile config x K split, with and without dX (2560x1568, K 1024) in
the same launch.  us per launch (events, mean of 30), relative error vs float64 once per config.

    python tools/wgrad_probe.py
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
    return round(e0.elapsed_time(e1) / n * 1000.0, 1)


def main():
    g = torch.Generator(device=DEV).manual_seed(0)
    Kr = 2560
    dg = torch.randn(Kr, 1024, generator=g, device=DEV)      # dgates rows (time-major)
    dz = torch.randn(Kr, 512, generator=g, device=DEV)
    h = torch.randn(Kr, 256, generator=g, device=DEV)
    x = torch.randn(Kr, 1568, generator=g, device=DEV)
    w = torch.randn(1024, 1568, generator=g, device=DEV) * 0.02
    dgh, dgl = split(dg)
    dzh, dzl = split(dz)
    hh, hl = split(h)
    xh, xl = split(x)
    wh, wl = split(w)
    ws = torch.zeros(64 << 20, device=DEV)
    tk = torch.zeros(4096, dtype=torch.int32, device=DEV)
    probs = [Gemm(dzh.t(), hh, torch.zeros(512, 256, device=DEV), a_lo=dzl.t(), b_lo=hl),
             Gemm(dgh.t(), hh, torch.zeros(1024, 256, device=DEV), a_lo=dgl.t(), b_lo=hl),
             Gemm(dgh.t(), xh, torch.zeros(1024, 1568, device=DEV), a_lo=dgl.t(), b_lo=xl)]
    refs = [dz.double().t() @ h.double(), dg.double().t() @ h.double(), dg.double().t() @ x.double()]
    dxc = torch.empty(Kr, 1568, dtype=torch.bfloat16, device=DEV)
    dx = Gemm(dgh, wh, dxc, a_lo=dgl, b_lo=wl, c_lo=torch.empty_like(dxc))
    out = {}
    for cfg, (bm, bn, bk, ns) in enumerate(G5_CFGS):
        if bm % 128 or bn % 128:
            continue
        for s in (1, 2, 3, 4, 6, 8):
            def run(with_dx=False, s=s, cfg=cfg):
                for p in probs:
                    p.c.zero_()
                ps = probs + ([dx] if with_dx else [])
                gemm_sp(ps, splits=[s, s, s] + ([1] if with_dx else []), cfg=cfg, ws=ws, tickets=tk)
            key = f"{bm}x{bn}x{bk}/{ns} s{s}"
            try:
                run()
            except Exception as e:   # noqa: BLE001
                out[key] = str(e)[:80]
                continue
            torch.cuda.synchronize()
            err = max(((p.c.double() - r).norm() / r.norm()).item() for p, r in zip(probs, refs))
            out[key] = {"w_us": timeit(run), "w_dx_us": timeit(lambda: run(True)), "relerr": f"{err:.1e}"}
            print(key, json.dumps(out[key]), flush=True)
    # the whole group on the 128-wide tiles with dX split too
    for cfg in (1, 6):
        for s in (2, 3, 4):
            for sx in (2, 3, 4):
                def run2(s=s, sx=sx, cfg=cfg):
                    for p in probs:
                        p.c.zero_()
                    gemm_sp(probs + [dx], splits=[s, s, s, sx], cfg=cfg, ws=ws, tickets=tk)
                key = f"{G5_CFGS[cfg]} s{s} dx s{sx}"
                out[key] = timeit(run2)
                print(key, out[key], flush=True)


if __name__ == "__main__":
    main()
