"""Debug: tagged BPTT vs counter BPTT per time step (fast and sc1 paths)."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from test_kernels_gpu import _setup, _rel, UNITS  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402
DEV = "cuda"
for B, H in ((8, 256), (64, 256)):
    cfg, net, L, flat, pk = _setup(B, H, seed=1)
    T, t0, G = 9, 3, 4 * H
    k = kernels()
    gates = torch.rand(T - t0, B, G, device=DEV)
    cseq = torch.randn(T, B, H, device=DEV)
    c0 = torch.randn(B, H, device=DEV)
    dh_ext = torch.randn(T - t0, B, H, device=DEV)
    ctr = torch.zeros(int(k.r2_lstm_persist_ctr_words()), dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    slab = torch.zeros(2, H // UNITS, B, H, device=DEV)
    dg_ref = torch.zeros(T - t0, B, G, dtype=torch.bfloat16, device=DEV)
    k.r2_lstm_bwd_persist(ptr(dh_ext), ptr(gates), ptr(cseq), ptr(c0), ptr(pk["w_hhT"]), ptr(slab),
                          ptr(dg_ref), B, T, t0, H, ptr(ctr), ptr(err), stream_handle())
    ring = torch.full((k.r2_lstm_bwd_tag_ring_bytes(B, H) // 4,), -1, dtype=torch.int32, device=DEV)
    for slow in (0, 1):
        k.r2_lstm_persist_force_slow(slow)
        dg = torch.zeros_like(dg_ref)
        k.r2_lstm_bwd_tag(ptr(dh_ext), ptr(gates), ptr(cseq), ptr(c0), ptr(pk["w_hhT"]), ptr(dg),
                          B, T, t0, H, ptr(ctr), ptr(err), ptr(ring), 0, 0, 0, 0, *([0] * 15), stream_handle())
        torch.cuda.synchronize()
        print(B, H, "slow", slow, "err", err.item(), [round(_rel(dg[i].float(), dg_ref[i].float()), 4) for i in range(T - t0)])
        # per gate block error at tl = T - t0 - 2
        i = T - t0 - 2
        print("  per-gate", [round(_rel(dg[i, :, q::4].float(), dg_ref[i, :, q::4].float()), 4) for q in range(4)],
              "per 64-col block", [round(_rel(dg[i, :, 64 * q:64 * q + 64].float(), dg_ref[i, :, 64 * q:64 * q + 64].float()), 3) for q in range(4)])
    k.r2_lstm_persist_force_slow(0)
