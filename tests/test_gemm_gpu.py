"""Batched MFMA GEMM (csrc/kernels/gemm.hip) vs fp32 torch on bf16-rounded operands: all four
operand layouts, ragged edges, bias, output row map, accumulate, bf16 output, multi-problem."""
import pytest
import torch

from pytorch_r2d2_amd.ops.gemm import Gemm, gemm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.fixture(params=[2, 5, 6, 7, 8], ids=["v1v2", "v4_256x64", "v4_256x32", "v4_128x64", "v4_128x32"])
def gemm_version(request):
    """2: 128x128 kernels (register-staged / LDS-DMA by K); 5..8: the 8-wave 256 x BN x BK kernels."""
    from pytorch_r2d2_amd.ops._lib import kernels
    kernels().r2_gemm_set_version(request.param)
    yield request.param
    kernels().r2_gemm_set_version(2)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _op(rows, cols, kmajor, gen):
    """A (rows, cols) bf16 view that is row-contiguous (kmajor: cols = K contiguous) or
    column-contiguous."""
    x = torch.randn(rows, cols, generator=gen, device=DEV).bfloat16()
    return x if kmajor else x.t().contiguous().t()


@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("M,N,K", [(296, 200, 64), (1024, 1568, 96), (136, 264, 1568), (64, 48, 40),
                                   (520, 1568, 2560), (200, 136, 128), (5440, 1024, 1568), (2560, 1568, 1024)])
def test_gemm_layouts(ak, bk, M, N, K, gemm_version):
    """K % 64 == 0 runs the LDS-DMA kernel (v2), other K the register-staged one (v1); version 5
    runs every K % 8 == 0 shape on the 256x256 kernel (zero-block K tail)."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K + 2 * ak + bk)
    a = _op(M, K, ak, g)
    b = _op(N, K, bk, g).t()          # (K, N) view; k-major means B^T rows contiguous
    c = torch.empty(M, N, device=DEV)
    bias = torch.randn(N, generator=g, device=DEV)
    gemm(Gemm(a, b, c, bias=bias, alpha=0.5))
    torch.cuda.synchronize()
    ref = 0.5 * (a.float() @ b.float()) + bias
    assert _rel(c, ref) < 1e-5


def test_gemm_row_map_accumulate_bf16_and_batch(gemm_version):
    g = torch.Generator(device=DEV).manual_seed(3)
    M, N, K = 256, 1568, 128
    a = _op(K, M, 1, g).t()             # mn-major A (like dgates^T)
    b = _op(N, K, 0, g).t()             # mn-major B (like X)
    perm = torch.randperm(M, generator=torch.Generator().manual_seed(0)).to(DEV, torch.int32)
    c = torch.randn(M, N, generator=g, device=DEV)
    c0 = c.clone()
    a2 = _op(K, 64, 1, g).t()
    b2 = _op(256, K, 0, g).t()
    c2 = torch.empty(64, 256, dtype=torch.bfloat16, device=DEV)
    gemm(Gemm(a, b, c, crow=perm, accumulate=True), Gemm(a2, b2, c2))
    torch.cuda.synchronize()
    ref = c0.clone()
    ref[perm.long()] += a.float() @ b.float()
    assert _rel(c, ref) < 1e-5
    assert _rel(c2, a2.float() @ b2.float()) < 1e-2


@pytest.mark.parametrize("ak,bk", [(1, 1), (0, 0), (1, 0)])
def test_gemm_v1_v2_agree(ak, bk):
    from pytorch_r2d2_amd.ops._lib import kernels
    g = torch.Generator(device=DEV).manual_seed(11)
    M, N, K = 384, 512, 640
    a = _op(M, K, ak, g)
    b = _op(N, K, bk, g).t()
    outs = []
    for v in (1, 2):
        kernels().r2_gemm_set_version(v)
        c = torch.empty(M, N, device=DEV)
        gemm(Gemm(a, b, c))
        outs.append(c)
    kernels().r2_gemm_set_version(2)
    torch.cuda.synchronize()
    assert _rel(outs[0], outs[1]) < 1e-6


def test_gemm_group_split_k_deterministic():
    """gemm_group_kernel: k-major and mn-major A in one grid, K split 1/2/3 ways with the
    last-arriver reduction; bit-identical across runs (tickets self-reset) and vs fp32 torch."""
    from pytorch_r2d2_amd.ops.gemm import gemm_group, group_ws_bytes
    g = torch.Generator(device=DEV).manual_seed(21)
    probs, refs = [], []
    shapes = [(1024, 1568, 2560, 0, 2), (1024, 256, 2560, 0, 3), (520, 1568, 1024, 1, 1)]
    for M, N, K, ak, _ in shapes:
        a = _op(M, K, ak, g) if ak else _op(K, M, 1, g).t()
        b = _op(N, K, 0, g).t()
        c = torch.randn(M, N, generator=g, device=DEV)
        refs.append((c.clone(), a, b))
        probs.append(Gemm(a, b, c, accumulate=True))
    splits = [s[4] for s in shapes]
    ws = torch.zeros(group_ws_bytes(probs, splits) // 4 + 1, device=DEV)
    tickets = torch.zeros(1024, dtype=torch.int32, device=DEV)
    outs = []
    for _ in range(2):
        for p, (c0, _, _) in zip(probs, refs):
            p.c.copy_(c0)
        gemm_group(probs, splits, ws, tickets)
        torch.cuda.synchronize()
        outs.append([p.c.clone() for p in probs])
    assert int(tickets.abs().sum()) == 0
    for i, (c0, a, b) in enumerate(refs):
        assert torch.equal(outs[0][i], outs[1][i])
        assert _rel(outs[0][i], c0 + a.float() @ b.float()) < 1e-5
