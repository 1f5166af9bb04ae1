"""Is the split x-projection bound per workgroup or by a shared resource?  The 192x256 tile
(gemm_sp.hip cfg 7) at M pairs giving 128 / 192 / 224 (the bench shape) / 256 workgroups, one round
each: per-workgroup bound -> the same time at every count; aggregate bound -> time grows with it.
  python tools/xproj_wg_scaling.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm_sp  # noqa: E402

bf = torch.bfloat16
K, N = 1568, 1024
g = torch.Generator(device="cuda").manual_seed(0)


def split(x):
    h = x.to(bf)
    return h, (x - h.float()).to(bf)


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


W = [split(torch.randn(N, K, generator=g, device="cuda") * 0.02) for _ in range(2)]
bias = torch.randn(N, generator=g, device="cuda")
ws = torch.zeros(1, device="cuda")
tk = torch.zeros(4096, dtype=torch.int32, device="cuda")
res = {}
for ms in ((3072, 3072), (4608, 4608), (5440, 5120), (6144, 6144)):
    X = [split(torch.relu(torch.randn(m, K, generator=g, device="cuda"))) for m in ms]
    out = [torch.empty(m, N, device="cuda") for m in ms]
    pr = [Gemm(X[i][0], W[i][0].t(), out[i], bias=bias, a_lo=X[i][1], b_lo=W[i][1].t()) for i in range(2)]
    wgs = sum(-(-m // 192) for m in ms) * (N // 256)
    res["%d+%d (%d wg)" % (ms[0], ms[1], wgs)] = [timeit(lambda: gemm_sp(pr, cfg=7, ws=ws, tickets=tk))
                                                  for _ in range(3)]
print(json.dumps(res))
