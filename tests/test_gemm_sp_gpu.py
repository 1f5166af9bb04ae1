"""Fused split-precision GEMM (csrc/kernels/gemm_sp.hip) vs float64 PyTorch: every operand
layout, every tile shape, one- and two-plane operands, split outputs, row maps, accumulate,
grouped problems with K splits."""
import pytest
import torch

from pytorch_r2d2_amd.ops.gemm import G5_CFGS, Gemm, gemm_sp

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")

CFGS = list(range(len(G5_CFGS)))


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-300)).item()


def _split(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def _op(rows, cols, kmajor, gen):
    x = torch.randn(rows, cols, generator=gen, device=DEV)
    return x if kmajor else x.t().contiguous().t()


def _valid(ak, bk, cfg):
    bm, bn = G5_CFGS[cfg][:2]
    return not ((bm % 128 and not ak) or (bn % 128 and not bk))


@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 0), (0, 1)])
@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("M,N,K", [(5440, 1024, 1568), (304, 200, 128), (2560, 256, 512)])
def test_gemm_sp_fp32_accurate(ak, bk, cfg, M, N, K):
    if not _valid(ak, bk, cfg):
        pytest.skip("tile / layout combination not built")
    g = torch.Generator(device=DEV).manual_seed(M + N + K + ak + 2 * bk)
    a = _op(M, K, ak, g)
    b = _op(N, K, bk, g).t()
    ah, al = _split(a)
    bh, bl = _split(b)
    c = torch.empty(M, N, device=DEV)
    bias = torch.randn(N, generator=g, device=DEV)
    assert gemm_sp([Gemm(ah, bh, c, bias=bias, a_lo=al, b_lo=bl)], cfg=cfg) == cfg
    ref = a.double() @ b.double() + bias.double()
    torch.cuda.synchronize()
    r = _rel(c, ref)
    assert r < 2e-5, r


def test_gemm_sp_one_plane_split_output_rowmap_accumulate_group():
    g = torch.Generator(device=DEV).manual_seed(3)
    # split hi / lo output
    M, N, K = 1000, 320, 448
    a = _op(M, K, 1, g)
    ah0, al0 = _split(a)
    b = _op(N, K, 0, g).t()
    bh, bl = _split(b)
    ch = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    cl = torch.empty_like(ch)
    gemm_sp([Gemm(ah0, bh, ch, a_lo=al0, b_lo=bl, c_lo=cl)])
    ref = a.double() @ b.double()
    torch.cuda.synchronize()
    assert _rel(ch.double() + cl.double(), ref) < 2e-5
    # row map + accumulate into fp32
    perm = torch.randperm(M, generator=torch.Generator().manual_seed(1)).to(DEV, torch.int32)
    base = torch.randn(M, N, generator=g, device=DEV)
    c = base.clone()
    ah, al = _split(a * 1.5)
    gemm_sp([Gemm(ah, bh, c, crow=perm, accumulate=True, a_lo=al, b_lo=bl, alpha=0.5)])
    ref2 = base.double().clone()
    ref2[perm.long()] += 0.5 * ((a.double() * 1.5) @ b.double())
    torch.cuda.synchronize()
    assert _rel(c, ref2) < 2e-5
    # group: the learner's post-BPTT products (mn-major A dW problems + the k-major A dX
    # problem, mn-major B), K split 1..3 ways, in one launch
    probs, refs = [], []
    for (M, N, K, ak) in [(1024, 1568, 2560, 0), (1024, 256, 2560, 0), (512, 256, 2560, 0),
                          (2560, 1568, 1024, 1)]:
        x = _op(M, K, 1, g) if ak else _op(K, M, 1, g).t()
        y = _op(N, K, 0, g).t()
        xh, xl = _split(x)
        yh, yl = _split(y)
        c = torch.zeros(M, N, device=DEV)
        probs.append(Gemm(xh, yh, c, a_lo=xl, b_lo=yl))
        refs.append(x.double() @ y.double())
    for splits in ([1, 1, 1, 1], [3, 2, 2, 1]):
        for cfg in (1, 2, 3, -1):
            for p in probs:
                p.c.zero_()
            gemm_sp(probs, splits=splits, cfg=cfg)
            torch.cuda.synchronize()
            for p, r in zip(probs, refs):
                assert _rel(p.c, r) < 2e-5, (splits, cfg)
