"""One GEMM configuration, repeated: a target for rocprofv3 --pmc passes (tools/pmc_gemm.sh)."""
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops._lib import kernels  # noqa: E402
from pytorch_r2d2_amd.ops.gemm import Gemm, gemm  # noqa: E402

ver, reps = int(sys.argv[1]), int(sys.argv[2])
shape = sys.argv[3] if len(sys.argv) > 3 else "xp2"
torch.manual_seed(0)
bf = torch.bfloat16
X = (torch.rand(5440, 1568, device="cuda") * 2 - 1).to(bf)
X2 = (torch.rand(5440, 1568, device="cuda") * 2 - 1).to(bf)
W = (torch.rand(1024, 1568, device="cuda") * 2 - 1).to(bf)
C = torch.empty(5440, 1024, device="cuda")
C2 = torch.empty(5440, 1024, device="cuda")
dg = (torch.rand(2560, 1024, device="cuda") * 2 - 1).to(bf)
Cw = torch.empty(1024, 1568, device="cuda")
kernels().r2_gemm_set_version(ver)
for _ in range(reps):
    if shape == "xp2":
        gemm(Gemm(X, W.t(), C), Gemm(X2, W.t(), C2))
    else:
        gemm(Gemm(dg.t(), X[:2560], Cw))
torch.cuda.synchronize()
