"""x-projection of both nets (5440 / 5120 x 1568 . 1568 x 1024, fp32 out + bias, the 192x256 split
tile, gemm_sp.hip) under the mainloop variants and the decomposition probe instances
(r2_gemm5_set_mode bits 8-9): full, staging_only (no fragment reads, no MFMAs), compute_only (no
staging).  Interleaved rounds in one process, us per launch.
  python tools/xproj_decomp.py [rounds]"""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm_sp  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels  # noqa: E402

bf = torch.bfloat16
K, N = 1568, 1024
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
g = torch.Generator(device="cuda").manual_seed(0)


def split(x):
    h = x.to(bf)
    return h, (x - h.float()).to(bf)


X = [torch.relu(torch.randn(M, K, generator=g, device="cuda")) for M in (5440, 5120)]
W = [torch.randn(N, K, generator=g, device="cuda") * 0.02 for _ in range(2)]
bias = torch.randn(N, generator=g, device="cuda")
XS, WS = [split(x) for x in X], [split(w) for w in W]
out = [[torch.empty(x.shape[0], N, device="cuda") for x in X] for _ in range(2)]
probs = [[Gemm(XS[i][0], WS[i][0].t(), out[v][i], bias=bias, a_lo=XS[i][1], b_lo=WS[i][1].t())
          for i in range(2)] for v in range(2)]
ws = torch.zeros(1, device="cuda")
tk = torch.zeros(4096, dtype=torch.int32, device="cuda")
k = kernels()


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


modes = {"full": 0, "staging_only": 1 << 8, "compute_only": 2 << 8}
res = {m: [] for m in modes}
for _ in range(rounds):
    for m, bits in modes.items():
        k.r2_gemm5_set_mode(bits)
        res[m].append(timeit(lambda: gemm_sp(probs[0], cfg=7, ws=ws, tickets=tk)))
k.r2_gemm5_set_mode(0)
gemm_sp(probs[0], cfg=7, ws=ws, tickets=tk)
torch.cuda.synchronize()
ref = X[0].double() @ W[0].double().t() + bias.double()
res["rel_err"] = ((out[0][0].double() - ref).norm() / ref.norm()).item()
print(json.dumps(res))
