"""Why does the split x-projection take ~120 us inside the learner step but ~97 us back to back
(tools/xproj_wg_scaling.py)?  The bench-shape launch (5440 + 5120 rows, 192x256 tile) timed per rep
(events around it, no host sync between reps) after: nothing (warm), a 512 MB scratch write (cold MALL / L2, dirty lines), a 64 MB rewrite
of its own A operand (A just produced, as the torso kernel leaves it).  Medians of 30 reps, us.
  python tools/xproj_cold_probe.py"""
import json
import statistics
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


W = [split(torch.randn(N, K, generator=g, device="cuda") * 0.02) for _ in range(2)]
bias = torch.randn(N, generator=g, device="cuda")
ws = torch.zeros(1, device="cuda")
tk = torch.zeros(4096, dtype=torch.int32, device="cuda")
X = [split(torch.relu(torch.randn(m, K, generator=g, device="cuda"))) for m in (5440, 5120)]
out = [torch.empty(x[0].shape[0], N, device="cuda") for x in X]
pr = [Gemm(X[i][0], W[i][0].t(), out[i], bias=bias, a_lo=X[i][1], b_lo=W[i][1].t()) for i in range(2)]
scratch = torch.empty(128 * 1024 * 1024, dtype=torch.float32, device="cuda")
src = [(x[0].clone(), x[1].clone()) for x in X]


def pre_none():
    pass


def pre_scratch():
    scratch.fill_(1.0)


def pre_rewrite_a():
    for (h, lo), (sh, sl) in zip(X, src):
        h.copy_(sh)
        lo.copy_(sl)


res = {}
for name, pre in (("warm", pre_none), ("after_512MB_write", pre_scratch), ("after_A_rewrite", pre_rewrite_a),
                  ("warm2", pre_none)):
    evs = []
    for _ in range(35):   # no host sync between reps: the GPU stays busy (clocks steady)
        pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gemm_sp(pr, cfg=7, ws=ws, tickets=tk)
        e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize()
    ts = [a.elapsed_time(b) * 1e3 for a, b in evs]
    res[name] = round(statistics.median(ts[5:]), 1)
print(json.dumps(res))
