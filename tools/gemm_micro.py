"""MFMA GEMM (csrc/kernels/gemm.hip) vs torch/hipBLASLt at the learner step's shapes."""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


res = {}
bf = torch.bfloat16
# x-projection: (5440 x 1568) @ (1568 x 1024) + bias, fp32 out
X = torch.randn(5440, 1568, device=DEV).to(bf)
W = torch.randn(1024, 1568, device=DEV).to(bf)
bias = torch.randn(1024, device=DEV)
C = torch.empty(5440, 1024, device=DEV)
fl = 2 * 5440 * 1568 * 1024
us = timeit(lambda: gemm(Gemm(X, W.t(), C, bias=bias)))
res["xp_mine_us"], res["xp_mine_tflops"] = us, fl / us / 1e6
us = timeit(lambda: torch.addmm(bias, X, W.t(), out_dtype=torch.float32))
res["xp_torch_us"], res["xp_torch_tflops"] = us, fl / us / 1e6
# dW_ih: dgates^T (1024 x 2560) @ X (2560 x 1568), both mn-major
dg = torch.randn(2560, 1024, device=DEV).to(bf)
Xl = X[:2560]
Cw = torch.empty(1024, 1568, device=DEV)
fl = 2 * 1024 * 2560 * 1568
us = timeit(lambda: gemm(Gemm(dg.t(), Xl, Cw)))
res["dwih_mine_us"], res["dwih_mine_tflops"] = us, fl / us / 1e6
us = timeit(lambda: torch.mm(dg.t(), Xl, out_dtype=torch.float32))
res["dwih_torch_us"] = us
# dX: dgates (2560 x 1024) @ W (1024 x 1568) bf16 out (k-major A, mn-major B)
Cx = torch.empty(2560, 1568, dtype=bf, device=DEV)
us = timeit(lambda: gemm(Gemm(dg, W, Cx)))
res["dx_mine_us"], res["dx_mine_tflops"] = us, fl / us / 1e6
us = timeit(lambda: torch.mm(dg, W))
res["dx_torch_us"] = us
# v1 (register staged) vs v2 (LDS-DMA) on K % 64 shapes
from pytorch_r2d2_amd.ops._lib import kernels  # noqa: E402
Xp = torch.randn(5440, 1600, device=DEV).to(bf)
Wp = torch.randn(1024, 1600, device=DEV).to(bf)
fl = 2 * 5440 * 1600 * 1024
for v in (1, 2):
    kernels().r2_gemm_set_version(v)
    us = timeit(lambda: gemm(Gemm(Xp, Wp.t(), C, bias=bias)))
    res[f"xp1600_v{v}_us"], res[f"xp1600_v{v}_tflops"] = us, fl / us / 1e6
    us = timeit(lambda: gemm(Gemm(dg.t(), Xl, Cw)))
    res[f"dwih_v{v}_us"] = us
    us = timeit(lambda: gemm(Gemm(dg, W, Cx)))
    res[f"dx_v{v}_us"] = us
# v3/v4 at the step's real K (1568: K % 16 path)
for v in (2, 5, 7):
    kernels().r2_gemm_set_version(v)
    us = timeit(lambda: gemm(Gemm(X, W.t(), C, bias=bias)))
    res[f"xp_v{v}_us"] = us
    X2 = torch.randn(5440, 1568, device=DEV).to(bf)
    C2 = torch.empty(5440, 1024, device=DEV)
    us = timeit(lambda: gemm(Gemm(X, W.t(), C, bias=bias), Gemm(X2, W.t(), C2, bias=bias)))
    res[f"xp2net_v{v}_us"] = us
    err = (C - (X.float() @ W.float().t() + bias)).abs().max().item()
    res[f"xp_v{v}_maxerr"] = err
    us = timeit(lambda: gemm(Gemm(dg.t(), Xl, Cw)))
    res[f"dwih_v{v}_us"] = us
    err = (Cw - dg.float().t() @ Xl.float()).abs().max().item()
    res[f"dwih_v{v}_maxerr"] = err
    us = timeit(lambda: gemm(Gemm(dg, W, Cx)))
    res[f"dx_v{v}_us"] = us
kernels().r2_gemm_set_version(2)
print(json.dumps({k: round(v, 1) for k, v in res.items()}))
