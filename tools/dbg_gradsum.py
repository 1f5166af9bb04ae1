"""Debug probe for gradsum.hip head_grads: structured inputs, prints outputs and partials."""
import sys
sys.path.insert(0, ".")
import torch  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle  # noqa: E402

k = kernels()
DEV = "cuda"
N, A, HD = 128, 6, 256
W = 1 + A
for name, dva in (("ones", torch.ones(N, W, device=DEV)),
                  ("colidx", torch.arange(W, device=DEV).float().repeat(N, 1)),
                  ("rowidx", torch.arange(N, device=DEV).float()[:, None].repeat(1, W))):
    zr = torch.ones(N, 2 * HD, device=DEV).bfloat16()
    dz = torch.ones(N, 2 * HD, device=DEV).bfloat16()
    ws = torch.zeros(int(k.r2_gradsum_ws_floats()), device=DEV)
    ticket = torch.zeros(64, dtype=torch.int32, device=DEV)
    gw2 = torch.full((W, HD), float("nan"), device=DEV)
    gb2 = torch.full((W,), float("nan"), device=DEV)
    gb1 = torch.full((2 * HD,), float("nan"), device=DEV)
    k.r2_head_grads(ptr(dva), ptr(zr), ptr(dz), ptr(gw2), ptr(gb2), ptr(gb1), N, A, HD, ptr(ws),
                    ptr(ticket), stream_handle())
    torch.cuda.synchronize()
    print(name, "gw2", gw2[:, :4].tolist())
    print(name, "ref", (dva.t() @ zr.float())[:, :4].tolist())
    print(name, "gb2", gb2.tolist(), "gb1[:4]", gb1[:4].tolist())
    print(name, "ws blk0 col0", ws[:12].tolist())
    print(name, "ws blk0 col1", ws[12:24].tolist())
