"""Micro-benchmark of the fused TD / dueling-head kernel (td.hip td_duel_kernel) at the paper
config's shapes (Tl 40 x B 64 transitions, 6 actions, head hidden 256, split precision), random
data, events timing, per fusion variant:

  plain   TD + dueling backward only
  dh      + dh = dz @ W1 (the BPTT input gradient)
  fwd_dh  + the three heads' dueling forward (the engine's paper-config launch)

    python tools/td_micro.py [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402

DEV = torch.device("cuda")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
Tl, B, A, HD, H, Lb, cap = 40, 64, 6, 256, 256, 40, 1_000_000
n = Tl * B
g = torch.Generator(device=DEV).manual_seed(0)


def rnd(*s, scale=1.0):
    return torch.randn(*s, device=DEV, generator=g) * scale


q = [rnd(n, A) for _ in range(3)]
starts = torch.randint(0, cap - 200, (B,), dtype=torch.int32, device=DEV, generator=g)
probs = torch.rand(B, device=DEV, generator=g) * 1e-5 + 1e-6
action = torch.randint(0, A, (cap,), dtype=torch.uint8, device=DEV, generator=g)
reward = rnd(cap)
done = (torch.rand(cap, device=DEV, generator=g) < 0.01).to(torch.uint8)
dq = torch.empty(n, A, device=DEV)
loss = torch.empty(1, device=DEV)
td_abs = torch.empty(n, device=DEV)
prio = torch.zeros(cap, device=DEV)
is_w = torch.empty(B, device=DEV)
n_valid = torch.tensor([cap // 80], dtype=torch.int32, device=DEV)
part = torch.zeros(4096, device=DEV)
ticket = torch.zeros(4, dtype=torch.int32, device=DEV)
zr = rnd(n, 2 * HD)
w2 = rnd(1 + A, HD, scale=0.05)
dz = torch.empty(n, 2 * HD, dtype=torch.bfloat16, device=DEV)
dz_lo = torch.empty_like(dz)
dva = torch.empty(n, 1 + A, device=DEV)
w1t = rnd(H, 2 * HD, scale=0.05).to(torch.bfloat16)
w1t_lo = rnd(H, 2 * HD, scale=0.0005).to(torch.bfloat16)
dh = torch.empty(n, H, device=DEV)
zs = [rnd(n, 2 * HD) for _ in range(3)]
b1 = [rnd(2 * HD, scale=0.1) for _ in range(2)]
w2t = rnd(1 + A, HD, scale=0.05)
b2 = [rnd(1 + A, scale=0.1) for _ in range(2)]
qo = [torch.empty(n, A, device=DEV) for _ in range(3)]
fwd = np.asarray([ptr(zs[0]), ptr(zs[1]), ptr(zs[2]), ptr(b1[0]), ptr(b1[1]), ptr(w2t), ptr(b2[0]),
                  ptr(b2[1]), ptr(qo[0]), ptr(qo[1]), ptr(qo[2]), 0], dtype=np.int64)
k = kernels()


def launch(fuse_dh, fuse_fwd):
    def f():
        if fuse_fwd:
            k.r2_td_duel_fwd_set(fwd.ctypes.data)
        rc = k.r2_td_duel_dh(ptr(q[0]), ptr(q[1]), ptr(q[2]), ptr(starts), ptr(probs), ptr(action),
                             ptr(reward), ptr(done), ptr(dq), ptr(loss), ptr(td_abs), ptr(prio),
                             ptr(is_w), ptr(n_valid), Tl, B, A, Lb, cap, 0.997 ** 5, 1, 1e-3, 0.9,
                             1e-6, 0.6, ptr(part), ptr(ticket), ptr(zr), ptr(w2), ptr(dz), ptr(dva),
                             HD, ptr(dz_lo), 0, ptr(w1t) if fuse_dh else 0,
                             ptr(w1t_lo) if fuse_dh else 0, ptr(dh) if fuse_dh else 0, H,
                             stream_handle())
        assert rc == 0, rc
    return f


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


res = {name: timeit(launch(d, f_)) for name, d, f_ in
       (("plain", False, False), ("dh", True, False), ("fwd_dh", True, True))}
# stage stamps of the engine's launch: per-stage median / max over waves (us), and the spread
# of workgroup start times
tr = torch.zeros((n + 15) // 16, 16, 12, dtype=torch.int64, device=DEV)
k.r2_td_duel_set_trace(ptr(tr))
launch(True, True)()
torch.cuda.synchronize()
k.r2_td_duel_set_trace(None)
t = tr.cpu().numpy().astype(np.float64) / 100.0      # s_memrealtime: 100 MHz -> us
t0 = t[:, :, 0].min()
stages = {}
# stamp order in the kernel: 0 top, 1 staging issued, 2 after barrier 1, 8 heads forward done,
# 9 TD done, 3 dz stored, 4 after barrier 2, 5 dh done, 6 last flag, 7 loss (last workgroup)
seq = [(0, 1, "issue"), (1, 2, "barrier1"), (2, 8, "heads_fwd"), (8, 9, "td"), (9, 3, "dz"),
       (3, 4, "barrier2"), (4, 5, "dh"), (5, 6, "last_flag")]
for a_, b_, nm in seq:
    d = t[:, :, b_] - t[:, :, a_]
    stages[nm] = [round(float(np.median(d)), 2), round(float(d.max()), 2)]
stages["wg_start_spread"] = round(float(t[:, 0, 0].max() - t0), 2)
stages["wave_end_max"] = round(float(t[:, :, 6].max() - t0), 2)
stages["last_wg_end"] = round(float(t[:, :, 7].max() - t0), 2)
print(json.dumps({"td_duel_us": res, "stages_med_max_us": stages}))
