"""Which phase of the fp32 torso forward owns its LDS bank conflicts?  Runs torso_fwd_sp2_kernel at
the bench shape (tools/sp_micro.py's 4-job split over 10560 frames) under the timing-probe bits
(r2_torso_sp_debug: 1 skips conv1, 2 conv2, 4 conv3, 16 the next-frame staging, 64 the act1 save),
3 launches per variant, in a fixed order; ``--summarize`` reads the rocprofv3 counter CSV and
prints the per-variant means (dispatches in launch order).

    rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES \\
        --kernel-trace --output-format csv -d gpurun_out/tlds -- python tools/torso_lds_variants.py
    python tools/torso_lds_variants.py --summarize 'gpurun_out/tlds/*/*counter_collection.csv'
"""
import collections
import csv
import glob
import json
import os
import sys

VARIANTS = [(0, "full"), (1, "no_conv1"), (2, "no_conv2"), (4, "no_conv3"), (16, "no_frame"),
            (64, "no_save"), (1 | 4, "conv2_alone"), (2 | 4, "conv1_alone")]
PER = 3


def run():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import numpy as np
    import torch
    from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    B, T, n, Lb = 64, 80, 5, 40
    cap = 200_000
    frames = torch.randint(0, 256, (cap, 4 * 84 * 84), dtype=torch.uint8, device=dev, generator=g)

    def split(x):
        hi = x.to(torch.bfloat16)
        return hi, (x - hi.float()).to(torch.bfloat16)

    def net():
        w = [split(torch.randn(32, k, device=dev, generator=g) * 0.05) for k in (256, 512, 288)]
        b = [torch.randn(32, device=dev, generator=g) * 0.1 for _ in range(3)]
        return w, b

    (on_w, on_b), (tg_w, tg_b) = net(), net()
    # the job table of tools/sp_micro.py (TS_JOB_WORDS = 20 words per job)
    rows = torch.randint(0, cap, ((T + n) * B,), dtype=torch.int32, device=dev, generator=g)
    Xo = torch.empty(2, (T + n) * B, 1568, dtype=torch.bfloat16, device=dev)
    Xt = torch.empty(2, T * B, 1568, dtype=torch.bfloat16, device=dev)
    NL = (T - Lb) * B
    s1 = torch.empty(2, NL, 400, 32, dtype=torch.bfloat16, device=dev)
    s2 = torch.empty(2, NL, 81, 32, dtype=torch.bfloat16, device=dev)

    def job(w, b, r, X, save):
        z = 0
        return [ptr(r), r.numel(), ptr(w[0][0]), ptr(w[0][1]), ptr(b[0]), ptr(w[1][0]), ptr(w[1][1]),
                ptr(b[1]), ptr(w[2][0]), ptr(w[2][1]), ptr(b[2]), ptr(X[0]), ptr(X[1]),
                ptr(s1[0]) if save else z, ptr(s1[1]) if save else z,
                ptr(s2[0]) if save else z, ptr(s2[1]) if save else z, 0, 0, 0]

    jobs = np.asarray([
        job(on_w, on_b, rows[: Lb * B], Xo[:, : Lb * B], False),
        job(on_w, on_b, rows[Lb * B: T * B], Xo[:, Lb * B: T * B], True),
        job(on_w, on_b, rows[T * B:], Xo[:, T * B:], False),
        job(tg_w, tg_b, rows[n * B:], Xt, False)], dtype=np.int64)
    assert jobs.shape == (4, 20)
    k = kernels()
    n_cus = torch.cuda.get_device_properties(0).multi_processor_count
    for bits, _ in VARIANTS:
        k.r2_torso_sp_debug(bits)
        for _ in range(PER):
            assert k.r2_torso_fwd_sp_multi(ptr(frames), jobs.ctypes.data, 4, n_cus, stream_handle()) == 0
        torch.cuda.synchronize()
    k.r2_torso_sp_debug(0)
    print(json.dumps({"variants": [v for _, v in VARIANTS], "per": PER}))


def summarize(pattern):
    paths = sorted(glob.glob(pattern), key=os.path.getmtime)
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(paths[-1])):
        if "torso_fwd_sp2_kernel" in r["Kernel_Name"]:
            d = by[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ids = sorted(by)
    for vi, (_, name) in enumerate(VARIANTS):
        chunk = [by[d] for d in ids[vi * PER:(vi + 1) * PER]]
        if not chunk:
            continue
        mean = {c: sum(x.get(c, 0.0) for x in chunk) / len(chunk) for c in chunk[0]}
        conf, act = mean.get("SQ_LDS_BANK_CONFLICT", 0), mean.get("SQ_LDS_IDX_ACTIVE", 1)
        print(json.dumps({"variant": name, **{c: f"{v:.3e}" for c, v in mean.items()},
                          "conflict_over_active": round(conf / max(act, 1), 3)}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
