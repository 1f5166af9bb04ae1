"""Micro-benchmark of the split-precision (fp32-accurate) hot kernels at the atari57 fixed-mode
bench shapes, random data, events timing:

  torso   torso_fwd_sp_kernel over 10560 frames (online 85 + target 80 per sequence, B=64), the
          engine's 4-job split (burn-in / learning frames with activation saves / tail / target)
  xproj   fused split GEMM of both nets' x-projections (M 5440 / 5120, N 1024, K 1568)

    python tools/sp_micro.py {torso|xproj|both} [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm_sp  # noqa: E402

DEV = torch.device("cuda")
which = sys.argv[1] if len(sys.argv) > 1 else "both"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
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


def split(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


g = torch.Generator(device=DEV).manual_seed(0)
if which in ("torso", "both"):
    B, T, n, Lb = 64, 80, 5, 40
    cap = 200_000
    frames = torch.randint(0, 256, (cap, 4 * 84 * 84), dtype=torch.uint8, device=DEV, generator=g)
    rows = torch.randint(0, cap, ((T + n) * B,), dtype=torch.int32, device=DEV, generator=g)

    def net():
        w = [split(torch.randn(32, k, device=DEV, generator=g) * 0.05) for k in (256, 512, 288)]
        b = [torch.randn(32, device=DEV, generator=g) * 0.1 for _ in range(3)]
        return w, b

    (on_w, on_b), (tg_w, tg_b) = net(), net()
    Xo = torch.empty(2, (T + n) * B, 1568, dtype=torch.bfloat16, device=DEV)
    Xt = torch.empty(2, T * B, 1568, dtype=torch.bfloat16, device=DEV)
    NL = (T - Lb) * B
    s1 = torch.empty(2, NL, 400, 32, dtype=torch.bfloat16, device=DEV)
    s2 = torch.empty(2, NL, 81, 32, dtype=torch.bfloat16, device=DEV)

    def job(w, b, r, X, save):
        z = 0
        return [ptr(r), r.numel(), ptr(w[0][0]), ptr(w[0][1]), ptr(b[0]), ptr(w[1][0]), ptr(w[1][1]),
                ptr(b[1]), ptr(w[2][0]), ptr(w[2][1]), ptr(b[2]), ptr(X[0]), ptr(X[1]),
                ptr(s1[0]) if save else z, ptr(s1[1]) if save else z,
                ptr(s2[0]) if save else z, ptr(s2[1]) if save else z, 0, 0, 0]

    jobs = np.asarray([
        job(on_w, on_b, rows[: Lb * B], Xo[:, : Lb * B], False),
        job(on_w, on_b, rows[Lb * B: T * B], Xo[:, Lb * B: T * B], True),
        job(on_w, on_b, rows[T * B:], Xo[:, T * B:], False),
        job(tg_w, tg_b, rows[n * B:], Xt, False)], dtype=np.int64)
    k = kernels()
    n_cus = torch.cuda.get_device_properties(0).multi_processor_count
    res["torso_fwd_sp_us_10560"] = timeit(lambda: k.r2_torso_fwd_sp_multi(
        ptr(frames), jobs.ctypes.data, 4, n_cus, stream_handle()))
    if "probe" in sys.argv:
        # phase costs: skip conv1 / conv2 / conv3 (timing only) etc.; variants interleaved over 7
        # rounds, min of the per-round means (single back-to-back timings drift by +-15 %)
        variants = ((0, "full"), (1, "no_conv1"), (2, "no_conv2"), (4, "no_conv3"),
                    (7, "none"), (16, "no_frame"), (64, "no_save"), (119, "nothing"),
                    (1 | 4, "conv2_alone"))
        best = {}
        for _ in range(7):
            for bits, name in variants:
                k.r2_torso_sp_debug(bits)
                t = timeit(lambda: k.r2_torso_fwd_sp_multi(ptr(frames), jobs.ctypes.data, 4, n_cus,
                                                           stream_handle()))
                best[name] = min(best.get(name, 1e30), t)
        k.r2_torso_sp_debug(0)
        res.update({f"torso_{k_}_us": round(v, 1) for k_, v in best.items()})
        tr = torch.zeros(8 * 16 * 5, dtype=torch.int64, device=DEV)
        k.r2_torso_sp_trace(ptr(tr))
        k.r2_torso_fwd_sp_multi(ptr(frames), jobs.ctypes.data, 4, n_cus, stream_handle())
        torch.cuda.synchronize()
        k.r2_torso_sp_trace(0)
        t = tr.view(8, 16, 5).cpu()
        t0 = t[0, 2, 0].item()
        # cycles relative to frame 2's loop top of wave 0, frames 2..9
        res["trace_cycles_wave_frame_stamp"] = (t[:, 2:10] - t0).tolist()
        rows.zero_()
        res["torso_hot_frame_us"] = timeit(lambda: k.r2_torso_fwd_sp_multi(
            ptr(frames), jobs.ctypes.data, 4, n_cus, stream_handle()))
if which in ("xproj", "both"):
    xp = []
    for M in (5440, 5120):
        a, b = torch.randn(M, 1568, device=DEV, generator=g), torch.randn(1024, 1568, device=DEV, generator=g).t()
        ah, al = split(a)
        bh, bl = split(b)
        xp.append(Gemm(ah, bh, torch.empty(M, 1024, device=DEV), bias=torch.randn(1024, device=DEV),
                       a_lo=al, b_lo=bl))
    res["xproj_cfg"] = gemm_sp(xp)
    res["xproj_us"] = timeit(lambda: gemm_sp(xp))
    if "probe" in sys.argv:
        probs = []
        for (M, N, K, ak) in [(1024, 1568, 2560, 0), (1024, 256, 2560, 0), (512, 256, 2560, 0),
                              (2560, 1568, 1024, 1)]:
            x = torch.randn(M, K, device=DEV, generator=g) if ak else \
                torch.randn(K, M, device=DEV, generator=g).t()
            y = torch.randn(N, K, device=DEV, generator=g).t().contiguous()
            xh, xl = split(x)
            yh, yl = split(y)
            probs.append(Gemm(xh, yh, torch.zeros(M, N, device=DEV), a_lo=xl, b_lo=yl))
        for c in (0, 1, 3, 6):
            res[f"xproj_cfg{c}_us"] = timeit(lambda: gemm_sp(xp, cfg=c))
        for c in (1, 3, 6):
            res[f"group_cfg{c}_us"] = timeit(lambda: gemm_sp(probs, splits=[4, 4, 4, 1], cfg=c))
print(json.dumps(res))
