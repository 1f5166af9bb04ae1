"""x-projection GEMM of both nets (atari57: 5440 x 1568 . 1568 x 1024, fp32 out + bias) under
each forced 8-wave kernel variant (gemm.hip r2_gemm_set_version) and hipBLASLt."""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels  # noqa: E402

bf = torch.bfloat16
M, D, G = 5440, 1568, 1024
X = [torch.randn(M, D, device="cuda").to(bf) for _ in range(2)]
W = [torch.randn(G, D, device="cuda").to(bf) for _ in range(2)]
bias = torch.randn(G, device="cuda")
out = [torch.empty(M, G, device="cuda") for _ in range(2)]


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)


res = {}
ref = X[0].float() @ W[0].float().t() + bias
for v in (2, 5, 6, 7, 8):
    kernels().r2_gemm_set_version(v)
    res[f"v{v}"] = timeit(lambda: gemm(*[Gemm(X[i], W[i].t(), out[i], bias=bias) for i in range(2)]))
    res[f"v{v}_err"] = ((out[0] - ref).norm() / ref.norm()).item()
kernels().r2_gemm_set_version(2)
res["torch"] = timeit(lambda: [torch.addmm(bias, X[i], W[i].t(), out_dtype=torch.float32) for i in range(2)])
print(json.dumps(res))
