"""fp32 (split) torso backward at the bench shape (2560 learning frames): time and the per-stage
clock stamps of workgroup 0 (S0 inputs -> LDS, S1 g2 on waves 5-7, S2 dW2 + g1, S2b frame, S3 dW1)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402

DEV = "cuda"
k = kernels()
g = torch.Generator(device=DEV).manual_seed(0)
n, cap = 2560, 100_000
frames = torch.randint(0, 256, (cap, 28224), dtype=torch.uint8, device=DEV, generator=g)
rows = torch.randint(0, cap, (n,), dtype=torch.int32, device=DEV, generator=g)


def bf(*shape, relu=False):
    x = torch.randn(*shape, device=DEV, generator=g)
    return (x.relu() if relu else x).bfloat16()


a1, a1l, a2, a2l = bf(n, 400, 32, relu=True), bf(n, 400, 32), bf(n, 81, 32, relu=True), bf(n, 81, 32)
dx, dxl, o3 = bf(n, 1568), bf(n, 1568), bf(n, 1568, relu=True)
w3, w3l, w2, w2l = bf(32, 288), bf(32, 288), bf(4, 32, 128), bf(4, 32, 128)
grid = torch.cuda.get_device_properties(0).multi_processor_count
slab = torch.zeros(grid * int(k.r2_torso_bwd_slab_floats()), device=DEV)
nsl = int(k.r2_torso_bwd_slab_floats())
dst = torch.arange(nsl, dtype=torch.int32, device=DEV)
scale = torch.ones(nsl, device=DEV)
grad = torch.zeros(nsl, device=DEV)
run = lambda: k.r2_torso_bwd_sp(ptr(frames), ptr(rows), n, ptr(a1), ptr(a1l), ptr(a2), ptr(a2l), ptr(dx),
                                ptr(dxl), ptr(o3), ptr(w3), ptr(w3l), ptr(w2), ptr(w2l), ptr(slab), grid,
                                ptr(dst), ptr(scale), ptr(grad), stream_handle())
res = {}
assert run() == 0
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    run()
e1.record()
torch.cuda.synchronize()
res["bwd_sp_us"] = e0.elapsed_time(e1) / 10 * 1e3
tr = torch.zeros(8 * 16 * 11, dtype=torch.int64, device=DEV)
k.r2_torso_bwd_sp_trace(ptr(tr))
run()
torch.cuda.synchronize()
k.r2_torso_bwd_sp_trace(0)
t = tr.view(8, 16, 11).cpu()
stages = []
for fi in range(1, 8):
    row = [int(t[:, fi, j + 1].max() - t[:, fi, j].max()) for j in range(5)]
    row.append(int(t[:, fi + 1, 0].max() - t[:, fi, 5].max()))
    stages.append(row)
res["stage_cycles_S0_S1_S2_S2b_S3_loop"] = stages
res["median"] = [int(np.median([r[j] for r in stages])) for j in range(6)]
# S2 split: dW2 part per wave (from the S1 barrier to the wave's stamp 6), dact1 part
res["S2_dW2_cycles_per_wave"] = [int(t[w, 3, 6] - t[:, 3, 2].max()) for w in range(8)]
res["S2_dact1_cycles_per_wave"] = [int(t[w, 3, 3] - t[w, 3, 6]) for w in range(8)]
# dact1 split per wave: K loop (stamp 6 -> 7), epilogue + next-frame prefetch issue (7 -> 8),
# barrier wait (8 -> 3)
res["S2_dact1_kloop_epi_barrier_per_wave"] = [[int(t[w, 3, 7] - t[w, 3, 6]), int(t[w, 3, 8] - t[w, 3, 7]),
                                               int(t[w, 3, 3] - t[w, 3, 8])] for w in range(8)]
# S1 per wave (waves 0-5): tap loop (stamp 1 -> 9), epilogue + db2 reduction (9 -> 10), barrier (10 -> 2)
res["S1_loop_epi_barrier_per_wave"] = [[int(t[w, 3, 9] - t[w, 3, 1]), int(t[w, 3, 10] - t[w, 3, 9]),
                                        int(t[w, 3, 2] - t[w, 3, 10])] for w in range(6)]
for bits in (1, 2, 3):
    k.r2_torso_bwd_sp_debug(bits)
    run()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    res[f"bwd_sp_us_dbg{bits}"] = e0.elapsed_time(e1) / 10 * 1e3
k.r2_torso_bwd_sp_debug(0)
print(json.dumps(res))
