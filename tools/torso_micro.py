"""Micro-benchmark of the fused torso forward / backward kernels at the atari57 bench shapes
(fwd: 10880 frames = 2 nets x 64 x 85; bwd: 2560 learning frames), random data, events timing."""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.config import get_config  # noqa: E402
from pytorch_r2d2_amd.engine.layout import ParamLayout  # noqa: E402
from pytorch_r2d2_amd.models import QNet  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402

DEV = "cuda"
which = sys.argv[1] if len(sys.argv) > 1 else "both"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
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


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


if which in ("fwd", "both"):
    n = 10880
    rows = torch.randint(0, cap, (n,), dtype=torch.int32, device=DEV)
    out = torch.zeros(n, 1568, dtype=torch.bfloat16, device=DEV)
    res["torso_fwd_us_10880"] = timeit(lambda: k.r2_torso_fwd(
        ptr(frames), ptr(rows), n, ptr(pk["conv1"]), ptr(pk["b1"]), ptr(pk["conv2"]), ptr(pk["b2"]),
        ptr(pk["conv3"]), ptr(pk["b3"]), ptr(out), 0, 0, 256, stream_handle()))
if which in ("bwd", "both"):
    n = 2560
    rows = torch.randint(0, cap, (n,), dtype=torch.int32, device=DEV)
    a1 = torch.randn(n, 400, 32, device=DEV).relu().bfloat16()
    a2 = torch.randn(n, 81, 32, device=DEV).relu().bfloat16()
    dx = torch.randn(n, 1568, device=DEV).bfloat16()
    o3 = torch.randn(n, 1568, device=DEV).relu().bfloat16()
    grid = 256
    slab = torch.zeros(grid * int(k.r2_torso_bwd_slab_floats()), device=DEV)
    dst, scale = L.torso_grad_map()
    dst, scale = dst.to(DEV), scale.to(DEV)
    g = torch.zeros(L.padded, device=DEV)
    res["torso_bwd_us_2560"] = timeit(lambda: k.r2_torso_bwd(
        ptr(frames), ptr(rows), n, ptr(a1), ptr(a2), ptr(dx), ptr(o3), ptr(pk["conv3_dg"]),
        ptr(pk["conv2_dg"]), ptr(slab), grid, ptr(dst), ptr(scale), ptr(g), stream_handle()))
print(json.dumps(res))
