"""Split-precision GEMMs of one fp32 learner step: round-1 multi-pass kernels (gemm.hip gemm4 /
gemm_group) vs the fused one-pass kernel (gemm_sp.hip) on the engine's shapes, every tile.

    python tools/gemm_sp_micro.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_r2d2_amd.ops.gemm import G5_CFGS, Gemm, gemm, gemm_group, gemm_sp, group_ws_bytes  # noqa: E402

DEV = torch.device("cuda")


def split(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def op(rows, cols, kmajor, g):
    x = torch.randn(rows, cols, generator=g, device=DEV)
    return x if kmajor else x.t().contiguous().t()


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
    g = torch.Generator(device=DEV).manual_seed(0)
    out = {}
    # x-projection of both nets (fixed target mode, atari57): M 5440 / 5120, N 1024, K 1568
    xp = []
    for M in (5440, 5120):
        a, b = op(M, 1568, 1, g), op(1024, 1568, 1, g).t()
        ah, al = split(a)
        bh, bl = split(b)
        xp.append(Gemm(ah, bh, torch.empty(M, 1024, device=DEV), bias=torch.randn(1024, device=DEV),
                       a_lo=al, b_lo=bl))
    out["xproj_multipass_us"] = timeit(lambda: gemm(*xp))
    for c, cf in enumerate(G5_CFGS):
        out[f"xproj_fused_{'x'.join(map(str, cf))}_us"] = timeit(lambda: gemm_sp(xp, cfg=c))
    out["xproj_fused_auto_us"] = timeit(lambda: gemm_sp(xp))
    out["xproj_auto_cfg"] = gemm_sp(xp)
    # post-BPTT group: dW_ih, dW_hh, dW_head1 (mn-major A), dX (k-major A, split output)
    probs = []
    for (M, N, K, ak) in [(1024, 1568, 2560, 0), (1024, 256, 2560, 0), (512, 256, 2560, 0),
                          (2560, 1568, 1024, 1)]:
        x = op(M, K, 1, g) if ak else op(K, M, 1, g).t()
        y = op(N, K, 0, g).t()
        xh, xl = split(x)
        yh, yl = split(y)
        if ak:
            ch = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            probs.append(Gemm(xh, yh, ch, a_lo=xl, b_lo=yl, c_lo=torch.empty_like(ch)))
        else:
            probs.append(Gemm(xh, yh, torch.zeros(M, N, device=DEV), a_lo=xl, b_lo=yl))
    ws = torch.zeros(group_ws_bytes(probs, [1, 1, 1, 1]) // 4 + 1, device=DEV)
    tk = torch.zeros(1024, dtype=torch.int32, device=DEV)
    out["group_multipass_us"] = timeit(lambda: gemm_group(probs, [1, 1, 1, 1], ws, tk))
    for splits in ([1, 1, 1, 1], [2, 2, 2, 1], [3, 2, 2, 1], [3, 3, 3, 1], [4, 4, 4, 1],
                   [4, 4, 4, 2], [5, 4, 4, 2]):
        for c in (1, 3, -1):
            key = f"group_fused_{'x'.join(map(str, splits))}_cfg{c}_us"
            out[key] = timeit(lambda: gemm_sp(probs, splits=splits, cfg=c))
    # heads (3 nets' first layers) and dh
    hs = []
    for rows in (2560, 2560, 2560):
        a, b = op(rows, 256, 1, g), op(512, 256, 1, g).t()
        ah, al = split(a)
        bh, bl = split(b)
        hs.append(Gemm(ah, bh, torch.empty(rows, 512, device=DEV), a_lo=al, b_lo=bl))
    out["heads_multipass_us"] = timeit(lambda: gemm(*hs))
    out["heads_fused_auto_us"] = timeit(lambda: gemm_sp(hs))
    for c in range(len(G5_CFGS)):
        out[f"heads_fused_cfg{c}_us"] = timeit(lambda: gemm_sp(hs, cfg=c))
    a, b = op(2560, 512, 1, g), op(256, 512, 0, g).t()
    ah, al = split(a)
    bh, bl = split(b)
    dh = [Gemm(ah, bh, torch.empty(2560, 256, device=DEV), a_lo=al, b_lo=bl)]
    out["dh_multipass_us"] = timeit(lambda: gemm(*dh))
    out["dh_fused_auto_us"] = timeit(lambda: gemm_sp(dh))
    for c in (0, 1, 2, 3):   # B (W_head1^T slice) is mn-major: BN=64 tiles are not built for it
        for sp in (1, 2, 4):
            out[f"dh_fused_cfg{c}_split{sp}_us"] = timeit(lambda: gemm_sp(dh, splits=[sp], cfg=c))
    print(json.dumps({k: round(v, 1) for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
