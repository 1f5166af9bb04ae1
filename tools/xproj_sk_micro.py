"""Split x-projection (bench shape, 192x256 tile): whole tiles (224 workgroups) vs the stream-K deal
(gemm_sp.hip gemm6_sk_kernel) over 256 / 240 / 232 workgroups, back-to-back launches, us.
  python tools/xproj_sk_micro.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops._lib import kernels, ptr  # noqa: E402
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm_sp  # noqa: E402

bf = torch.bfloat16
K, N = 1568, 1024
g = torch.Generator(device="cuda").manual_seed(0)


def split(x):
    h = x.to(bf)
    return h, (x - h.float()).to(bf)


X = [split(torch.relu(torch.randn(m, K, generator=g, device="cuda"))) for m in (5440, 5120)]
W = [split(torch.randn(N, K, generator=g, device="cuda") * 0.02) for _ in range(2)]
bias = torch.randn(N, generator=g, device="cuda")
out = [torch.empty(x[0].shape[0], N, device="cuda") for x in X]
pr = [Gemm(X[i][0], W[i][0].t(), out[i], bias=bias, a_lo=X[i][1], b_lo=W[i][1].t()) for i in range(2)]
ws = torch.zeros(2 * 224 * 192 * 256, device="cuda")
tk = torch.zeros(4096, dtype=torch.int32, device="cuda")
err = torch.zeros(1, dtype=torch.int32, device="cuda")
k = kernels()


def run(grid):
    if grid:
        k.r2_gemm5_set_sk(grid, ptr(err))
    gemm_sp(pr, cfg=7, ws=ws, tickets=tk, n_cus=256)


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
for _ in range(2):
    for grid in (0, 256, 240, 232):
        res.setdefault(str(grid or "whole"), []).append(timeit(lambda: run(grid)))
res["err"] = int(err.item())
print(json.dumps(res))
