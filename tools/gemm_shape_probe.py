"""Small-GEMM cost model probe: time the 128x128 MFMA GEMM (gemm.hip v2) at the head shapes
while sweeping K and the output dtype, to split a launch into a fixed part (prologue latency,
epilogue stores) and a per-K-tile part.  Compares torch.mm (hipBLASLt) at each point."""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels  # noqa: E402

DEV = "cuda"
bf = torch.bfloat16


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 2)


res = {}
kernels().r2_gemm_set_version(2)
for (M, N) in ((5760, 512), (2560, 256), (2560, 1024)):
    for K in (64, 128, 256, 512, 1024):
        A = torch.randn(M, K, device=DEV).to(bf)
        Bt = torch.randn(N, K, device=DEV).to(bf)
        Bm = torch.randn(K, N, device=DEV).to(bf)
        for cdt in ("bf16", "f32"):
            C = torch.empty(M, N, device=DEV, dtype=bf if cdt == "bf16" else torch.float32)
            res[f"M{M}_N{N}_K{K}_{cdt}_kk"] = timeit(lambda: gemm(Gemm(A, Bt.t(), C)))
            res[f"M{M}_N{N}_K{K}_{cdt}_km"] = timeit(lambda: gemm(Gemm(A, Bm, C)))
        res[f"M{M}_N{N}_K{K}_torch"] = timeit(lambda: torch.mm(A, Bm))
print(json.dumps(res))
