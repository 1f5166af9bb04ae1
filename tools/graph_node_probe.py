"""Per-kernel cost of a graph node vs an eager launch: the same tiny kernel (replay.hip
step_end_kernel) and a 1-tile GEMM, 50x eager and 50x as nodes of one HIP graph.  Run under
rocprofv3 --kernel-trace; the trace's per-dispatch durations split by phase."""
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402

bf = torch.bfloat16
step = torch.zeros(1, dtype=torch.int64, device="cuda")
dirty = torch.zeros(1, dtype=torch.int32, device="cuda")
A = torch.randn(128, 64, device="cuda").to(bf)
Bt = torch.randn(128, 64, device="cuda").to(bf)
C = torch.empty(128, 128, device="cuda")


def body():
    for _ in range(50):
        kernels().r2_step_end(ptr(step), ptr(dirty), stream_handle())
    for _ in range(50):
        gemm(Gemm(A, Bt.t(), C))


body()
torch.cuda.synchronize()
torch.cuda.nvtx.range_push("eager") if hasattr(torch.cuda, "nvtx") else None
body()
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
torch.cuda.synchronize()
for _ in range(2):
    g.replay()
torch.cuda.synchronize()
print("ok")
