"""Fixed per-launch cost of the 128x128 MFMA GEMM: one-tile and many-tile launches at K = 64,
an empty-ish kernel of the same library for the floor, and torch.mm for comparison.  Run under
rocprofv3 --kernel-trace --stats to separate kernel time from dispatch gaps."""
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402

bf = torch.bfloat16
dev = "cuda"
cases = {}
for (M, N, K) in ((128, 128, 64), (5760, 512, 64), (5760, 512, 256)):
    A = torch.randn(M, K, device=dev).to(bf)
    Bt = torch.randn(N, K, device=dev).to(bf)
    C = torch.empty(M, N, device=dev)
    cases[(M, N, K)] = (A, Bt, C)
step = torch.zeros(1, dtype=torch.int64, device=dev)
dirty = torch.zeros(1, dtype=torch.int32, device=dev)
for _ in range(20):
    for (M, N, K), (A, Bt, C) in cases.items():
        gemm(Gemm(A, Bt.t(), C))
        torch.mm(A, Bt.t())
    kernels().r2_step_end(ptr(step), ptr(dirty), stream_handle())
torch.cuda.synchronize()
print("ok")
