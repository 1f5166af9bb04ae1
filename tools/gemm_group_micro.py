"""Grouped split-K GEMM (gemm_group_kernel) vs the separate launches and hipBLASLt on the
learner's post-BPTT products (atari57 shapes)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm, gemm_group, group_ws_bytes  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)
bf = torch.bfloat16


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)


N, D, G, H, HD2 = 2560, 1568, 1024, 256, 512
X = torch.randn(N, D, device=DEV).to(bf)
Wih = torch.randn(G, D, device=DEV).to(bf)
dg = torch.randn(N, G, device=DEV).to(bf)
hseq = torch.randn(N, H, device=DEV).to(bf)
dz = torch.randn(N, HD2, device=DEV).to(bf)
dWih = torch.empty(G, D, device=DEV)
dWhh = torch.empty(G, H, device=DEV)
gw1 = torch.empty(HD2, H, device=DEV)
dX = torch.empty(N, D, dtype=bf, device=DEV)
P = {"wih": Gemm(dg.t(), X, dWih), "whh": Gemm(dg.t(), hseq, dWhh), "gw1": Gemm(dz.t(), hseq, gw1),
     "dx": Gemm(dg, Wih, dX)}
ws = torch.zeros(64 << 20, device=DEV)
tk = torch.zeros(4096, dtype=torch.int32, device=DEV)
res = {"sep_w3": timeit(lambda: gemm(P["wih"], P["whh"], P["gw1"])),
       "sep_wih": timeit(lambda: gemm(P["wih"])),
       "sep_dx": timeit(lambda: gemm(P["dx"])),
       "torch_wih": timeit(lambda: torch.mm(dg.t(), X, out_dtype=torch.float32)),
       "torch_dx": timeit(lambda: torch.mm(dg, Wih))}
cases = {"wih": [("wih",)], "dx": [("dx",)], "all": [("wih", "whh", "gw1", "dx")]}
for name, (probs,) in cases.items():
    for s in (1, 2, 3, 4, 5, 8):
        sp = [1 if p == "dx" else s for p in probs]
        if name == "dx":
            sp = [s]
        jobs = [P[p] for p in probs]
        assert group_ws_bytes(jobs, sp) <= ws.numel() * 4
        res[f"grp_{name}_s{s}"] = timeit(lambda: gemm_group(jobs, sp, ws, tk))
ref = dg.float().t() @ X.float()
gemm_group([P["wih"]], [4], ws, tk)
torch.cuda.synchronize()
res["grp_wih_s4_relerr"] = ((dWih - ref).norm() / ref.norm()).item()
print(json.dumps(res))
