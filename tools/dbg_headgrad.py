"""Debug: engine head-gradient path (fused gradsum vs torch) on the test_engine shape."""
import sys
sys.path.insert(0, ".")
import torch
sys.path.insert(0, "tests")
from test_engine_gpu import _make, _rel  # noqa
cfg, rp, eng, net, tgt = _make("shifted")
eng._forward_loss()
eng._backward_core()
torch.cuda.synchronize()
L = eng.layout
A, HD = L.A, L.HD
N = eng.Ll * eng.B
zr = eng.zr_on[:N].float()
g2 = eng.dva.t() @ zr
got = L.span(eng.grad, "val.2.weight", "adv.2.weight", (1 + A, HD))
print("val.2.w rel", _rel(got[0], g2[0, :HD]), "adv.2.w rel", _rel(got[1:], g2[1:, HD:]))
print("gb2 rel", _rel(L.span(eng.grad, "val.2.bias", "adv.2.bias", (1 + A,)), eng.dva.sum(0)))
print("gb1 rel", _rel(L.span(eng.grad, "val.0.bias", "adv.0.bias", (2 * HD,)), eng.dz.float().sum(0)))
print("got val2 norm", got[0].norm().item(), "ref", g2[0, :HD].norm().item())
print(got[0, :8], g2[0, :8])
