"""Measure how a HIP stream CU mask maps onto MI355X XCDs / CUs.

For each mask, a probe kernel (csrc/kernels/streams.hip cu_probe_kernel) records the XCC id and
HW_ID of every workgroup; we report how many distinct CUs of each XCD were used.

    python tools/cumask_probe.py > gpurun_out/cumask.txt
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ctypes  # noqa: E402

import torch  # noqa: E402

from pytorch_r2d2_amd.ops._lib import kernels  # noqa: E402


def probe(k, stream_h, nblocks=4096, spin=4):
    out = torch.zeros(2 * nblocks, dtype=torch.int32, device="cuda")
    rc = k.r2_cu_probe(ctypes.c_void_p(out.data_ptr()), nblocks, spin, ctypes.c_void_p(stream_h))
    assert rc == 0, rc
    torch.cuda.synchronize()
    v = out.view(nblocks, 2).cpu().tolist()
    per = collections.defaultdict(set)
    for xcc, hw in v:
        cu = (hw >> 8) & 15
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 7
        per[xcc].add((se, sh, cu))
    return {x: sorted(s) for x, s in sorted(per.items())}


def make_stream(k, words):
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    rc = k.r2_stream_create_cumask(arr, len(words), ctypes.byref(h))
    assert rc == 0, rc
    return h.value


def main():
    k = kernels()
    n_cus = torch.cuda.get_device_properties(0).multi_processor_count
    nw = (n_cus + 31) // 32
    print("CUs", n_cus, "words", nw)
    got = (ctypes.c_uint32 * nw)()
    print("default stream:")
    full = probe(k, torch.cuda.current_stream().cuda_stream)
    for x, s in full.items():
        print(f"  xcc {x}: {len(s)} CUs  e.g. {s[:6]}")
    masks = {
        "first 32 bits": [0xFFFFFFFF] + [0] * (nw - 1),
        "low 4 bits of every word": [0x0000000F] * nw,
        "every 8th bit": [0x01010101] * nw,
        "all but first 32 bits": [0] + [0xFFFFFFFF] * (nw - 1),
        "all but every 8th bit": [0xFEFEFEFE] * nw,
    }
    for name, words in masks.items():
        h = make_stream(k, words)
        k.r2_stream_get_cumask(ctypes.c_void_p(h), got, nw)
        res = probe(k, h)
        tot = sum(len(s) for s in res.values())
        print(f"mask {name}: {[hex(w) for w in words[:2]]}... readback {[hex(w) for w in got[:2]]}"
              f" -> {tot} CUs; per xcc " + ", ".join(f"{x}:{len(s)}" for x, s in res.items()))
        for x, s in res.items():
            print(f"    xcc {x}: {s}")
        k.r2_stream_destroy(ctypes.c_void_p(h))


if __name__ == "__main__":
    main()
