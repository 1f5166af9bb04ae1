"""dh = dz @ W1 (the head backward's 40-tile GEMM, M=2560 N=256 K=512, fp32 out): one launch of
the 128x128 kernel vs the grouped split-K launch (deterministic last-arriver reduce) vs
hipBLASLt, timed as 50 nodes of one HIP graph."""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm, gemm_group, group_ws_bytes  # noqa: E402

bf = torch.bfloat16
dz = torch.randn(2560, 512, device="cuda").to(bf)
w1 = torch.randn(512, 256, device="cuda").to(bf)
dh = torch.empty(2560, 256, device="cuda")


def timeit(fn, reps=50):
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


ref = dz.float() @ w1.float()
res = {"gemm": timeit(lambda: gemm(Gemm(dz, w1, dh)))}
res["gemm_err"] = ((dh - ref).norm() / ref.norm()).item()
for sp in (1, 2, 4, 8):
    p = Gemm(dz, w1, dh)
    ws = torch.zeros(max(group_ws_bytes([p], [sp]), 16) // 4, device="cuda")
    tk = torch.zeros(1024, dtype=torch.int32, device="cuda")
    res[f"group_s{sp}"] = timeit(lambda: gemm_group([p], [sp], ws, tk))
    res[f"group_s{sp}_err"] = ((dh - ref).norm() / ref.norm()).item()
res["torch_bf16out"] = timeit(lambda: torch.mm(dz, w1))
try:
    res["torch_f32out"] = timeit(lambda: torch.mm(dz, w1, out_dtype=torch.float32))
except Exception as e:  # noqa: BLE001
    res["torch_f32out"] = str(e)[:60]
print(json.dumps(res))
