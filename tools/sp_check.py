"""Print the fp32 (split precision) engine's per-tensor relative error vs a float64 oracle
(debug aid for tests/test_split_gpu.py)."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_split_gpu import _make, _oracle64, _rel  # noqa: E402

for mode in sys.argv[1:] or ["fixed"]:
    for dt in ("fp32", "bf16"):
        cfg, rp, eng, net, tgt = _make(mode, dtype=dt)
        eng._forward_loss()
        eng._backward_core()
        eng._backward_torso()
        torch.cuda.synchronize()
        online, out = _oracle64(rp, eng, net, tgt, cfg, mode)
        got = eng.layout.views(eng.grad)
        print(f"== {mode} {dt}: loss rel {abs(eng.loss.item() - out['loss'].item()) / out['loss'].item():.3e}")
        for n, p in online.named_parameters():
            print(f"   {n:24s} {_rel(got[n].cpu(), p.grad):.3e}")
