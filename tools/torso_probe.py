"""Diagnostics for the fused torso kernels: per-frame cost slope (n frames per workgroup) and
HBM sensitivity (all rows identical -> frames L2-resident).  Prints one JSON line."""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.config import get_config  # noqa: E402
from pytorch_r2d2_amd.engine.layout import ParamLayout  # noqa: E402
from pytorch_r2d2_amd.models import QNet  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402

DEV = "cuda"
k = kernels()
cfg = get_config("atari57")
torch.manual_seed(0)
L = ParamLayout(cfg.model, cfg.env)
flat = L.from_module(QNet("cpu", cfg.model, cfg.env), DEV)
bf = torch.zeros(L.bf_numel, dtype=torch.bfloat16, device=DEV)
f32 = torch.zeros(L.f_numel, device=DEV)
L.pack_torch(flat, bf, f32)
pk = L.packed_views(bf, f32)
cap = 200_000
frames = torch.randint(0, 256, (cap, 28224), dtype=torch.uint8, device=DEV)
res = {}


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps * 1e3, 1)


def fwd(n, same=False, grid=256):
    rows = (torch.zeros if same else lambda m, **kw: torch.randint(0, cap, (m,), **kw))(n, dtype=torch.int32, device=DEV)
    out = torch.zeros(n, 1568, dtype=torch.bfloat16, device=DEV)
    return timeit(lambda: k.r2_torso_fwd(
        ptr(frames), ptr(rows), n, ptr(pk["conv1"]), ptr(pk["b1"]), ptr(pk["conv2"]), ptr(pk["b2"]),
        ptr(pk["conv3"]), ptr(pk["b3"]), ptr(out), 0, 0, grid, stream_handle()))


for n in (256, 2560, 10880):
    res[f"fwd_n{n}"] = fwd(n)
res["fwd_n10880_same_row"] = fwd(10880, True)
res["fwd_n10880_grid128"] = fwd(10880, grid=128)

dst, scale = L.torso_grad_map()
dst, scale = dst.to(DEV), scale.to(DEV)
grad = torch.zeros(L.padded, device=DEV)


def bwd(n, same=False, grid=256):
    rows = (torch.zeros if same else lambda m, **kw: torch.randint(0, cap, (m,), **kw))(n, dtype=torch.int32, device=DEV)
    a1 = torch.randn(n, 400, 32, device=DEV).relu().bfloat16()
    a2 = torch.randn(n, 81, 32, device=DEV).relu().bfloat16()
    dx = torch.randn(n, 1568, device=DEV).bfloat16()
    o3 = torch.randn(n, 1568, device=DEV).relu().bfloat16()
    slab = torch.zeros(grid * int(k.r2_torso_bwd_slab_floats()), device=DEV)
    return timeit(lambda: k.r2_torso_bwd(
        ptr(frames), ptr(rows), n, ptr(a1), ptr(a2), ptr(dx), ptr(o3), ptr(pk["conv3_dg"]),
        ptr(pk["conv2_dg"]), ptr(slab), grid, ptr(dst), ptr(scale), ptr(grad), stream_handle()))


for n in (256, 1280, 2560):
    res[f"bwd_n{n}"] = bwd(n)
res["bwd_n2560_same_row"] = bwd(2560, True)
res["bwd_n2560_grid128"] = bwd(2560, grid=128)
print(json.dumps(res))

# per-phase clock trace of workgroup 0 (bwd, n=2560 -> 10 frames): S0 | S1 | S2 | S3 cycles
dbg = torch.zeros(16 * 8, dtype=torch.int64, device=DEV)
k.r2_torso_bwd_set_debug(ptr(dbg))
bwd(2560)
k.r2_torso_bwd_set_debug(None)
t = dbg.view(16, 8).cpu()
phases = []
for i in range(10):
    r = t[i]
    if r[0] == 0 or r[4] == 0:
        break
    phases.append([int(r[j + 1] - r[j]) for j in range(4)] +
                  [int(r[5] - r[2]), int(r[6] - r[5]), int(r[7] - r[6]), int(r[3] - r[7])])
print(json.dumps({"bwd_phase_cycles_S0_S1_S2_S3__S2split_pf_dw2_dact1_wait": phases}))

# forward: phase A (conv1 || conv3) | barrier wait | phase B (conv2, frame -> LDS) for frames of WG 0
dbg = torch.zeros(16 * 8, dtype=torch.int64, device=DEV)
k.r2_torso_fwd_set_debug(ptr(dbg))
fwd(10880)
k.r2_torso_fwd_set_debug(None)
t = dbg.view(16, 8).cpu()
ph = []
for i in range(15):
    if t[i + 1][0] == 0:
        break
    ph.append([int(t[i][1] - t[i][0]), int(t[i][2] - t[i][1]), int(t[i][4] - t[i][2]),
               int(t[i][5] - t[i][4]), int(t[i][6] - t[i][5]), int(t[i][3] - t[i][6])])
print(json.dumps({"fwd_phase_cycles_A_waitA_conv2mma_conv2epi_framewrite_waitB": ph}))
