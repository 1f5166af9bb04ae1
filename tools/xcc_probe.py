"""Block -> XCD placement of consecutive launches (is it b % 8, and from which XCD?)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.ops._lib import kernels, stream_handle  # noqa: E402

k = kernels()
res = {}
for name, nb, thr, lds in (("a256", 256, 256, 0), ("b128", 128, 256, 0), ("c7", 7, 64, 0),
                           ("d256", 256, 512, 150000), ("e256", 256, 256, 0), ("f13", 13, 64, 0),
                           ("g256", 256, 256, 0)):
    out = torch.full((nb,), -1, dtype=torch.int32, device="cuda")
    k.r2_xcc_probe(out.data_ptr(), nb, thr, lds, stream_handle())
    torch.cuda.synchronize()
    o = out.tolist()
    offs = sorted({(x - b) % 8 for b, x in enumerate(o)})
    res[name] = {"first16": o[:16], "offsets(xcc-b)%8": offs}
print(json.dumps(res))
