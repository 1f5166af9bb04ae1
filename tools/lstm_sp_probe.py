"""Persistent LSTM forward, split precision (4-byte tagged words = default, 8-byte granules) vs bf16, at the atari57 fixed-mode bench shape (H=256,
B=64, T=80, 3 chains): us/step and the per-step phase clock trace of workgroup (0,0,0):
[poll granules + hi/lo split, barrier, MFMA + gate exchange, pointwise, publish, to next step]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402

DEV = "cuda"
k = kernels()
H, G, B, T, NC = 256, 1024, 64, 80, 3
g = torch.Generator(device=DEV).manual_seed(0)
res = {}


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


nwg = H // 16
whh = (torch.randn(nwg, 64, H, device=DEV, generator=g) * 0.05)
whh_hi = whh.bfloat16()
whh_lo = (whh - whh_hi.float()).bfloat16()
xproj = torch.randn(T * B, G, device=DEV, generator=g)
c0 = torch.zeros(B, H, device=DEV)
err = torch.zeros(1, dtype=torch.int32, device=DEV)
keep = []


def site():   # one ctr + ring per launch site (the 4-bit tags of the sp hand-off need it)
    return (torch.zeros(int(k.r2_lstm_persist_ctr_words()), dtype=torch.int32, device=DEV),
            torch.zeros(k.r2_lstm_tag_ring_bytes(4, B, H) // 4, dtype=torch.int32, device=DEV))


def chains(sp, outs=None):
    out = []
    for c in range(NC):
        hs = torch.zeros(T, B, H, dtype=torch.bfloat16, device=DEV)
        hl = torch.zeros_like(hs)
        cs = torch.zeros(T, B, H, device=DEV)
        gt = torch.zeros(T, B, G, device=DEV)
        h0 = torch.zeros(B, H, device=DEV) if sp else torch.zeros(B, H, dtype=torch.bfloat16, device=DEV)
        keep.extend([hs, hl, cs, gt, h0])
        if outs is not None:
            outs.append((hs, hl, cs))
        d = [ptr(xproj), ptr(whh_hi), ptr(h0), ptr(c0), ptr(hs), ptr(cs), 0,
             ptr(gt) if c == 0 else 0, 40 if c == 0 else 0]
        if sp:
            d += [ptr(whh_lo), ptr(hl)]
        out.append(d)
    return np.asarray([v for ch in out for v in ch], dtype=np.int64)


o4, o8 = [], []
arr_sp, arr_sp8, arr_bf = chains(True, o4), chains(True, o8), chains(False)
s4, s8, sb = site(), site(), site()


def f_sp():
    k.r2_lstm_sp_handoff8(0)
    return k.r2_lstm_fwd_tag_sp(arr_sp.ctypes.data, NC, B, T, H, ptr(s4[0]), ptr(err), ptr(s4[1]), stream_handle())


def f_sp8():
    k.r2_lstm_sp_handoff8(1)
    rc = k.r2_lstm_fwd_tag_sp(arr_sp8.ctypes.data, NC, B, T, H, ptr(s8[0]), ptr(err), ptr(s8[1]), stream_handle())
    k.r2_lstm_sp_handoff8(0)
    return rc


f_bf = lambda: k.r2_lstm_fwd_tag(arr_bf.ctypes.data, NC, B, T, H, ptr(sb[0]), ptr(err), ptr(sb[1]), stream_handle())
res["sp_us_per_step"] = timeit(f_sp) / T
res["sp8_us_per_step"] = timeit(f_sp8) / T
res["bf16_us_per_step"] = timeit(f_bf) / T
torch.cuda.synchronize()
# 4-byte-word hand-off vs 8-byte granules: same recurrence up to the 2^-20 rounding of the words
dh = max(float(((a[0].double() + a[1].double()) - (b[0].double() + b[1].double())).abs().max()) for a, b in zip(o4, o8))
dc = max(float((a[2].double() - b[2].double()).abs().max()) for a, b in zip(o4, o8))
res["sp4_vs_sp8_max_abs_h"], res["sp4_vs_sp8_max_abs_c"] = dh, dc
res["c_max_abs"] = max(float(a[2].abs().max()) for a in o4)
for name, fn in (("sp", f_sp), ("sp8", f_sp8), ("bf16", f_bf)):
    dbg = torch.zeros(32 * 8 + 256, dtype=torch.int64, device=DEV)
    k.r2_lstm_persist_set_debug(ptr(dbg))
    fn()
    k.r2_lstm_persist_set_debug(None)
    torch.cuda.synchronize()
    t = dbg[:256].view(32, 8).cpu()
    rows = [[int(t[i][5] - t[i][0]), int(t[i][1] - t[i][5]), int(t[i][2] - t[i][1]),
             int(t[i][3] - t[i][2]), int(t[i][4] - t[i][3]), int(t[i + 1][0] - t[i][4])] for i in range(2, 14)]
    res[f"{name}_trace_poll_barrier_mma_pointwise_publish_next"] = rows
    res[f"{name}_trace_median"] = [int(np.median([r[j] for r in rows])) for j in range(6)]
res["err"] = int(err.item())
print(json.dumps(res))
