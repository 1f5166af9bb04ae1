"""Micro-benchmark: per-launch floor vs LSTM step kernels (eager and HIP-graph replay)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.config import get_config  # noqa: E402
from pytorch_r2d2_amd.engine.layout import ParamLayout, UNITS  # noqa: E402
from pytorch_r2d2_amd.models import QNet  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402

DEV = "cuda"
k = kernels()
k.r2_noop_chain.argtypes = [ctypes_p := __import__("ctypes").c_void_p, __import__("ctypes").c_int,
                            __import__("ctypes").c_int, ctypes_p]


def timeit(fn, reps=20, graph=False):
    if graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        run = g.replay
    else:
        run = fn
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


res = {}
cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
for blocks in (1, 32, 256):
    for graph in (False, True):
        us = timeit(lambda: k.r2_noop_chain(ptr(cnt), 100, blocks, stream_handle()), graph=graph)
        res[f"noop_x100_blocks{blocks}_{'graph' if graph else 'eager'}_us_per_launch"] = us / 100

cfg = get_config("atari57")
torch.manual_seed(0)
net = QNet("cpu", cfg.model, cfg.env)
L = ParamLayout(cfg.model, cfg.env)
flat = L.from_module(net, DEV)
bf = torch.zeros(L.bf_numel, dtype=torch.bfloat16, device=DEV)
f32 = torch.zeros(L.f_numel, device=DEV)
L.pack_torch(flat, bf, f32)
pk = L.packed_views(bf, f32)
H, G = 256, 1024
for B in (8, 64):
    T = 85
    xproj = torch.randn(T * B, G, device=DEV)
    h0 = torch.zeros(B, H, dtype=torch.bfloat16, device=DEV)
    c0 = torch.zeros(B, H, device=DEV)
    bufs = []
    chains = []
    for c in range(2):
        hs = torch.zeros(T, B, H, dtype=torch.bfloat16, device=DEV)
        cs = torch.zeros(T, B, H, device=DEV)
        gt = torch.zeros(T, B, G, device=DEV)
        bufs += [hs, cs, gt]
        chains.append([ptr(xproj), ptr(pk["w_hh"]), ptr(h0), ptr(c0), ptr(hs), ptr(cs), 0, ptr(gt), 40])
    ctr = torch.zeros(int(k.r2_lstm_persist_ctr_words()), dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    for nch in (1, 2):
        arr = np.asarray([v for ch in chains[:nch] for v in ch], dtype=np.int64)
        for graph in (False, True):
            us = timeit(lambda: k.r2_lstm_fwd(arr.ctypes.data, nch, B, T, H, 0, stream_handle()), graph=graph)
            res[f"lstm_fwd_B{B}_chains{nch}_{'graph' if graph else 'eager'}_us_per_step"] = us / T
            us = timeit(lambda: k.r2_lstm_fwd_persist(arr.ctypes.data, nch, B, T, H, ptr(ctr), ptr(err), stream_handle()), graph=graph)
            res[f"persist_fwd_B{B}_chains{nch}_{'graph' if graph else 'eager'}_us_per_step"] = us / T
    Tl = 40
    dh = torch.randn(Tl, B, H, device=DEV)
    s0 = torch.zeros(16, B, H, device=DEV)
    s1 = torch.zeros_like(s0)
    dc = torch.zeros(B, H, device=DEV)
    dg = torch.zeros(Tl, B, G, dtype=torch.bfloat16, device=DEV)
    gt = bufs[2]
    for graph in (False, True):
        us = timeit(lambda: k.r2_lstm_bwd(ptr(dh), ptr(gt), ptr(bufs[1]), ptr(c0), ptr(pk["w_hhT"]), ptr(s0), ptr(s1),
                                          ptr(dc), ptr(dg), B, 80, 40, H, stream_handle()), graph=graph)
        res[f"lstm_bwd_B{B}_{'graph' if graph else 'eager'}_us_per_step"] = us / 40
        slab = torch.zeros(2, 16, B, H, device=DEV)
        us = timeit(lambda: k.r2_lstm_bwd_persist(ptr(dh), ptr(gt), ptr(bufs[1]), ptr(c0), ptr(pk["w_hhT"]), ptr(slab),
                                                  ptr(dg), B, 80, 40, H, ptr(ctr), ptr(err), stream_handle()), graph=graph)
        res[f"persist_bwd_B{B}_{'graph' if graph else 'eager'}_us_per_step"] = us / 40
    torch.cuda.synchronize()
    res[f"persist_err_B{B}"] = int(err.item())
print(json.dumps(res, indent=1))
