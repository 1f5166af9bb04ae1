import json, sys, torch
sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm
bf = torch.bfloat16
def timeit(fn, reps=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)
dz = torch.randn(2560, 512, device="cuda").to(bf)
W1 = torch.randn(512, 256, device="cuda").to(bf)
dh = torch.empty(2560, 256, device="cuda")
h2 = [torch.randn(2880, 256, device="cuda").to(bf) for _ in range(2)]
z2 = [torch.empty(2880, 512, device="cuda", dtype=bf) for _ in range(2)]
r = {}
r["dh_mine"] = timeit(lambda: gemm(Gemm(dz, W1, dh)))
r["dh_torch"] = timeit(lambda: torch.mm(dz, W1, out_dtype=torch.float32))
r["head1_mine"] = timeit(lambda: gemm(*[Gemm(h2[i], W1.t(), z2[i]) for i in range(2)]))
r["head1_torch"] = timeit(lambda: [torch.mm(h2[i], W1.t(), out=z2[i]) for i in range(2)])
r["head1_torch_cat"] = timeit(lambda: torch.mm(torch.cat(h2), W1.t()))
print(json.dumps(r))
