"""How far is a plain fp32 PyTorch learner step (GPU and CPU) from the float64 one on the same
batch?  Calibrates the fp32-engine tolerance (tests/test_split_gpu.py)."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from tests.test_split_gpu import _make, _rel  # noqa: E402
from pytorch_r2d2_amd.learner_ref import batch_from_hbm, r2d2_loss  # noqa: E402

torch.backends.cudnn.allow_tf32 = False
torch.backends.cuda.matmul.allow_tf32 = False
mode = sys.argv[1] if len(sys.argv) > 1 else "fixed"
cfg, rp, eng, net, tgt = _make(mode, dtype="fp32")
eng._forward_loss()
torch.cuda.synchronize()
res = {}
for tag, dev, dt in (("fp64", "cpu", torch.float64), ("fp32cpu", "cpu", torch.float32),
                     ("fp32gpu", "cuda", torch.float32)):
    on = copy.deepcopy(net).to(dev, dt)
    tg = copy.deepcopy(tgt).to(dev, dt)
    b = batch_from_hbm(rp, eng.starts, eng.probs, cfg, dev)
    for f in ("obs", "h0", "c0", "th0", "tc0", "nh0", "nc0", "reward", "done", "weights"):
        v = getattr(b, f)
        if v is not None:
            setattr(b, f, v.to(dt))
    out = r2d2_loss(on, tg, b, cfg, mode)
    out["loss"].backward()
    res[tag] = (out["loss"].item(), {n: p.grad.detach().cpu().double() for n, p in on.named_parameters()})
l64, g64 = res["fp64"]
for tag in ("fp32cpu", "fp32gpu"):
    l, gg = res[tag]
    print(f"{tag}: loss rel {abs(l - l64) / abs(l64):.3e}  max grad rel {max(_rel(gg[n], g64[n]) for n in g64):.3e}")
    for n in g64:
        print(f"   {n:24s} {_rel(gg[n], g64[n]):.3e}")
