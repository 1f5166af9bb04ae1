"""Interference probe for verdict item 1 (x-projection on the LSTM forward's idle CUs): does the
recurrence slow down when a split GEMM of the x-projection's shape runs on the CUs its launch
leaves idle?

The fixed-target fp32 step's forward (lstm_persist.hip lstm_fwd_tag_launch, xcd_map 2) places 12
groups x 16 workgroups: XCDs 0-3 full (two groups), XCDs 4-7 half (one group) -> 64 idle CUs.
Here, per step of an eager engine, a side stream waits for the point right before the forward's
launch, sleeps ~10 us (the forward takes its CUs first), then queues ``--gemms`` x-projection-shaped
split GEMMs (both nets, 5440 / 5120 x 1568 . 1568 x 1024, 3 passes, 192 x 256 tiles): their
workgroups fill the free CUs while the recurrence runs.  Phases: alone / co-run / alone.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/corun -- python tools/xproj_corun_probe.py
    python tools/xproj_corun_probe.py --summarize 'gpurun_out/corun/*/*kernel_trace.csv'
"""
import argparse
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STEPS = 6


def run(n_gemms: int):
    import torch
    from pytorch_r2d2_amd.config import get_config
    from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    from pytorch_r2d2_amd.ops.gemm import Gemm, gemm_sp

    dev = torch.device("cuda")
    cfg = get_config("atari57", **{"seed": 1234, "learner.use_graph": False})
    replay = HBMReplay(cfg, dev, capacity=200_000)
    replay.fill_synthetic(episode_len=400, seed=0)
    eng = LearnerEngine(cfg, replay, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    xp = []
    for M in (5440, 5120):
        a = torch.randn(M, 1568, generator=g, device=dev)
        w = torch.randn(1024, 1568, generator=g, device=dev)
        ah, wh = a.to(torch.bfloat16), w.to(torch.bfloat16)
        xp.append(Gemm(ah, wh.t(), torch.empty(M, 1024, device=dev), bias=torch.zeros(1024, device=dev),
                       a_lo=(a - ah.float()).to(torch.bfloat16), b_lo=(w - wh.float()).to(torch.bfloat16).t()))
    side = torch.cuda.Stream()
    gemm_sp(xp, cfg=7)          # workspace / first-use setup outside the timed phases
    torch.cuda.synchronize()
    state = {"on": False}
    orig = eng._lstm

    def lstm(chains, T, t_begin=0, site=0):
        if state["on"] and T > 40:           # the main forward launch (not the reference nx site)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            side.wait_event(ev)
            with torch.cuda.stream(side):
                torch.cuda._sleep(20000)
                for _ in range(n_gemms):
                    gemm_sp(xp, cfg=7, stream=side.cuda_stream)
        return orig(chains, T, t_begin, site)

    eng._lstm = lstm
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    for phase in ("alone", "corun", "alone"):
        state["on"] = phase == "corun"
        for _ in range(STEPS):
            eng.step()
            torch.cuda.synchronize()
    print(json.dumps({"phases": ["warm x3", "alone", "corun", "alone"], "steps": STEPS,
                      "gemms": n_gemms, "error_word": int(eng.error_word())}), flush=True)


def summarize(pattern: str):
    paths = sorted(glob.glob(pattern), key=os.path.getmtime)
    rows = list(csv.DictReader(open(paths[-1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fwd = [r for r in rows if "lstm_fwd_tag_kernel" in r["Kernel_Name"]]
    bwd = [r for r in rows if "lstm_bwd_tag_kernel" in r["Kernel_Name"]]
    # the side stream's GEMMs: gemm6 192x256 launches on a queue other than the forward's
    q = fwd[0]["Queue_Id"]
    side = [r for r in rows if "gemm6_kernel<true, 192, 256" in r["Kernel_Name"] and r["Queue_Id"] != q]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3   # noqa: E731

    def overlap(r):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        cov = 0
        for o in side:
            a, b = max(s, int(o["Start_Timestamp"])), min(e, int(o["End_Timestamp"]))
            cov += max(0, b - a)
        return cov / max(1, e - s)

    out = []
    for i, r in enumerate(fwd):
        out.append({"i": i, "fwd_us": round(dur(r), 1), "side_gemm_overlap": round(overlap(r), 2),
                    "bptt_us": round(dur(bwd[i]), 1) if i < len(bwd) else None})
    for o in out:
        print(json.dumps(o))
    w = 3
    groups = {"alone_1": out[w:w + STEPS], "corun": out[w + STEPS:w + 2 * STEPS],
              "alone_2": out[w + 2 * STEPS:w + 3 * STEPS]}
    summ = {k: {"fwd_med_us": sorted(x["fwd_us"] for x in v)[len(v) // 2],
                "overlap_min": min(x["side_gemm_overlap"] for x in v)} for k, v in groups.items() if v}
    if side:
        summ["side_gemm_us_med"] = sorted(dur(o) for o in side)[len(side) // 2]
    print(json.dumps(summ))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemms", type=int, default=3)
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
    else:
        run(a.gemms)
