"""Round-6 verdict item 1 probe: does the BPTT tolerate target-net torso frames on the CUs it
leaves idle, and how many frames fit inside its window?

Eager engine steps (atari57 fp32 bench config).  In a co-run phase a side stream waits for the
point right before the BPTT launch (after the TD launch), sleeps ``--sleep`` cycles (the BPTT takes
its CUs first), then runs the split-precision torso forward (torso_fwd_sp2_kernel, target weights)
over the first M target-net frames of the step into a scratch buffer on ``--grid`` workgroups.
Phases: alone / co-run for each M / alone.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tcorun -- python tools/torso_bptt_corun_probe.py
    python tools/torso_bptt_corun_probe.py --summarize 'gpurun_out/tcorun/*/*kernel_trace.csv'
"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STEPS = 6


def run(frames_list, grid, sleep):
    import torch
    from pytorch_r2d2_amd.config import get_config
    from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    from pytorch_r2d2_amd.ops._lib import check, kernels, ptr

    dev = torch.device("cuda")
    cfg = get_config("atari57", **{"seed": 1234, "learner.use_graph": False})
    replay = HBMReplay(cfg, dev, capacity=200_000)
    replay.fill_synthetic(episode_len=400, seed=0)
    eng = LearnerEngine(cfg, replay, dev)
    side = torch.cuda.Stream()
    nmax = max(frames_list)
    out = torch.zeros(2, nmax, 1568, dtype=torch.bfloat16, device=dev)
    state = {"M": 0}
    orig = eng._backward_core_sp

    def bwd():
        M = state["M"]
        if M:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            side.wait_event(ev)
            rows = eng.rows[eng.t_lo_tg * eng.B:][:M]
            job = eng._torso_job_sp(eng.pk_t, eng.pk_t_lo, rows, out[0, :M], out[1, :M])
            state["job"] = np.asarray([job], dtype=np.int64)
            with torch.cuda.stream(side):
                if sleep:
                    torch.cuda._sleep(sleep)
                check(kernels().r2_torso_fwd_sp_multi(ptr(replay.frames), state["job"].ctypes.data, 1,
                                                      grid, side.cuda_stream), "side torso")
        return orig()

    eng._backward_core_sp = bwd
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    phases = [0] + list(frames_list) + [0]
    for M in phases:
        state["M"] = M
        for _ in range(STEPS):
            eng.step()
            torch.cuda.synchronize()
    print(json.dumps({"phases": phases, "steps": STEPS, "grid": grid, "sleep": sleep,
                      "error_word": int(eng.error_word())}), flush=True)


def summarize(pattern: str, phases):
    paths = sorted(glob.glob(pattern), key=os.path.getmtime)
    rows = list(csv.DictReader(open(paths[-1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    S = lambda r: int(r["Start_Timestamp"])   # noqa: E731
    E = lambda r: int(r["End_Timestamp"])     # noqa: E731
    bwd = [r for r in rows if "lstm_bwd_tag_kernel" in r["Kernel_Name"]]
    q = bwd[0]["Queue_Id"]
    main_torso = [r for r in rows if "torso_fwd_sp2" in r["Kernel_Name"] and r["Queue_Id"] == q]
    side = [r for r in rows if "torso_fwd_sp2" in r["Kernel_Name"] and r["Queue_Id"] != q]
    grp = [r for r in rows if "gemm6_kernel<false, 128, 128, 32>" in r["Kernel_Name"]]
    tb = [r for r in rows if "torso_bwd_sp_kernel" in r["Kernel_Name"]]
    res = []
    si = 0
    for i, b in enumerate(bwd):
        d = {"i": i, "bptt_us": round((E(b) - S(b)) / 1e3, 1)}
        if i < len(grp):
            d["group_us"] = round((E(grp[i]) - S(grp[i])) / 1e3, 1)
        if i < len(tb):
            d["torso_bwd_us"] = round((E(tb[i]) - S(tb[i])) / 1e3, 1)
        if i + 1 < len(main_torso):
            d["step_us"] = round((S(main_torso[i + 1]) - S(main_torso[i])) / 1e3, 1)
        if si < len(side) and S(side[si]) < E(b) + 5000 and S(side[si]) > S(b) - 50000:
            s = side[si]
            d["side_start_after_bptt_us"] = round((S(s) - S(b)) / 1e3, 1)
            d["side_end_after_bptt_end_us"] = round((E(s) - E(b)) / 1e3, 1)
            d["side_us"] = round((E(s) - S(s)) / 1e3, 1)
            si += 1
        res.append(d)
    for d in res:
        print(json.dumps(d))
    w = 3
    for pi, M in enumerate(phases):
        grp_ = res[w + pi * STEPS: w + (pi + 1) * STEPS]
        if not grp_:
            continue
        med = lambda k: sorted(x.get(k, 0) for x in grp_)[len(grp_) // 2]   # noqa: E731
        print(json.dumps({"phase": pi, "M": M, "bptt_med": med("bptt_us"), "group_med": med("group_us"),
                          "torso_bwd_med": med("torso_bwd_us"), "step_med": med("step_us"),
                          "side_end_after_bptt_end_med": med("side_end_after_bptt_end_us"),
                          "side_us_med": med("side_us")}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", default="768,1536,2304")
    ap.add_argument("--grid", type=int, default=192)
    ap.add_argument("--sleep", type=int, default=4000)
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    fl = [int(v) for v in a.frames.split(",")]
    if a.summarize:
        summarize(a.summarize, [0] + fl + [0])
    else:
        run(fl, a.grid, a.sleep)
