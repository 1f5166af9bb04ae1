"""The learner step's GEMM launches (shapes of the atari57 bench) under each kernel version."""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels  # noqa: E402

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
    return e0.elapsed_time(e1) / reps * 1e3


N, D, G, H, HD2 = 2560, 1568, 1024, 256, 512
X = torch.randn(5440, D, device=DEV).to(bf)
X2 = torch.randn(5440, D, device=DEV).to(bf)
Wih = torch.randn(G, D, device=DEV).to(bf)
bias = torch.randn(G, device=DEV)
xp1 = torch.empty(5440, G, device=DEV)
xp2 = torch.empty(5440, G, device=DEV)
dg = torch.randn(N, G, device=DEV).to(bf)
hseq = torch.randn(N, H, device=DEV).to(bf)
dz = torch.randn(N, HD2, device=DEV).to(bf)
head1 = torch.randn(HD2, H, device=DEV).to(bf)
dWih = torch.empty(G, D, device=DEV)
dWhh = torch.empty(G, H, device=DEV)
gw1 = torch.empty(HD2, H, device=DEV)
dX = torch.empty(N, D, dtype=bf, device=DEV)
dh = torch.empty(N, H, device=DEV)
zb = torch.empty(2880, HD2, dtype=bf, device=DEV)
hh = torch.randn(2880, H, device=DEV).to(bf)
jobs = {
    "xproj_2net": lambda: gemm(Gemm(X, Wih.t(), xp1, bias=bias), Gemm(X2, Wih.t(), xp2, bias=bias)),
    "dW_3prob": lambda: gemm(Gemm(dg.t(), X[:N], dWih), Gemm(dg.t(), hseq, dWhh), Gemm(dz.t(), hseq, gw1)),
    "dW_ih": lambda: gemm(Gemm(dg.t(), X[:N], dWih)),
    "dX": lambda: gemm(Gemm(dg, Wih, dX)),
    "dh": lambda: gemm(Gemm(dz, head1, dh)),
    "head1_fwd_2": lambda: gemm(Gemm(hh, head1.t(), zb), Gemm(hh, head1.t(), zb)),
}
refs = {}
res = {}
for v in (2, 9, 10, 5, 7):
    kernels().r2_gemm_set_version(v)
    for name, fn in jobs.items():
        try:
            res[f"{name}_v{v}"] = round(timeit(fn), 1)
        except RuntimeError as e:
            res[f"{name}_v{v}"] = str(e)[:40]
    fn = jobs["dW_ih"]
    fn()
    torch.cuda.synchronize()
    ref = dg.float().t() @ X[:N].float()
    res[f"dW_ih_v{v}_relerr"] = ((dWih - ref).norm() / ref.norm()).item()
    jobs["dX"]()
    torch.cuda.synchronize()
    ref = dg.float() @ Wih.float()
    res[f"dX_v{v}_relerr"] = ((dX.float() - ref).norm() / ref.norm()).item()
kernels().r2_gemm_set_version(2)
res["torch_dW_ih"] = round(timeit(lambda: torch.mm(dg.t(), X[:N], out_dtype=torch.float32)), 1)
res["torch_dX"] = round(timeit(lambda: torch.mm(dg, Wih)), 1)
print(json.dumps(res))
