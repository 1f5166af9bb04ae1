"""Persistent LSTM probe at the atari57 bench shape (H=256, B=64, T=85 fwd with 2 chains,
40-step BPTT): us/step and a per-step phase clock trace of workgroup (0,0,0) of the forward:
[xproj issue -> counter wait done, wait -> h loaded + MFMA + partials, pointwise, publish]."""
import json
import sys

import numpy as np
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
H, G, B, T = 256, 1024, 64, 85
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


xproj = torch.randn(T * B, G, device=DEV)
h0 = torch.zeros(B, H, dtype=torch.bfloat16, device=DEV)
c0 = torch.zeros(B, H, device=DEV)
bufs, chains = [], []
for c in range(2):
    hs = torch.zeros(T, B, H, dtype=torch.bfloat16, device=DEV)
    cs = torch.zeros(T, B, H, device=DEV)
    gt = torch.zeros(T, B, G, device=DEV)
    bufs += [hs, cs, gt]
    chains.append([ptr(xproj), ptr(pk["w_hh"]), ptr(h0), ptr(c0), ptr(hs), ptr(cs), 0, ptr(gt), 40])
ctr = torch.zeros(int(k.r2_lstm_persist_ctr_words()), dtype=torch.int32, device=DEV)
err = torch.zeros(1, dtype=torch.int32, device=DEV)
arr = np.asarray([v for ch in chains for v in ch], dtype=np.int64)
fwd_ctr = lambda: k.r2_lstm_fwd_persist(arr.ctypes.data, 2, B, T, H, ptr(ctr), ptr(err), stream_handle())
ring = torch.zeros(k.r2_lstm_tag_ring_bytes(2, B, H) // 4, dtype=torch.int32, device=DEV)
fwd_tag = lambda: k.r2_lstm_fwd_tag(arr.ctypes.data, 2, B, T, H, ptr(ctr), ptr(err), ptr(ring),
                                    stream_handle())
res["fwd_counter_us_per_step"] = timeit(fwd_ctr) / T
res["fwd_us_per_step"] = timeit(fwd_tag) / T
fwd = fwd_tag
dh = torch.randn(40, B, H, device=DEV)
slab = torch.zeros(2, 16, B, H, device=DEV)
dg = torch.zeros(40, B, G, dtype=torch.bfloat16, device=DEV)
bwd = lambda: k.r2_lstm_bwd_persist(ptr(dh), ptr(bufs[2]), ptr(bufs[1]), ptr(c0), ptr(pk["w_hhT"]), ptr(slab),
                                    ptr(dg), B, 80, 40, H, ptr(ctr), ptr(err), stream_handle())
res["bwd_counter_us_per_step"] = timeit(bwd) / 40
ring_b = torch.zeros(k.r2_lstm_bwd_tag_ring_bytes(B, H) // 4, dtype=torch.int32, device=DEV)
bwd_tag = lambda: k.r2_lstm_bwd_tag(ptr(dh), ptr(bufs[2]), ptr(bufs[1]), ptr(c0), ptr(pk["w_hhT"]),
                                    ptr(dg), B, 80, 40, H, ptr(ctr), ptr(err), ptr(ring_b), 0, 0, 0, 0, *([0] * 11),
                                    stream_handle())
res["bwd_us_per_step"] = timeit(bwd_tag) / 40
dbg = torch.zeros(32 * 8 + 256, dtype=torch.int64, device=DEV)
k.r2_lstm_persist_set_debug(ptr(dbg))
fwd()
k.r2_lstm_persist_set_debug(None)
torch.cuda.synchronize()
t = dbg[:256].view(32, 8).cpu()
res['blocks_g_xcc_fast'] = [int(v) - 1000 for v in dbg[256:].cpu() if v > 0]
res["fwd_trace_cycles_wait_mma_pointwise_publish_next"] = [
    [int(t[i][1] - t[i][0]), int(t[i][2] - t[i][1]), int(t[i][3] - t[i][2]), int(t[i][4] - t[i][3]),
     int(t[i + 1][0] - t[i][4])] for i in range(1, 12)]
res["fwd_trace_poll_barrier_ioarrive_minus_poll"] = [
    [int(t[i][5] - t[i][0]), int(t[i][1] - t[i][5]), int(t[i][6] - t[i][5])] for i in range(1, 12)]
res["err"] = int(err.item())
print(json.dumps(res))
