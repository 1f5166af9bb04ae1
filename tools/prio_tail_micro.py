"""Micro-timing of the learner's priority tail at the bench shape (B = 64 sequences of 80 + 5
rows, 64,000-row replay): the tail alone, the sample alone, and the hoisted step's fused tail +
next sample (replay.hip r2_prio_tail_sample), each launch bracketed by device events, medians of
``--reps`` launches.  Prints one JSON line.

    python tools/prio_tail_micro.py [--reps 50]
"""
import argparse
import json
import statistics

import torch

from pytorch_r2d2_amd.config import get_config
from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay

DEV = torch.device("cuda")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    cfg = get_config("atari57", **{"replay.capacity": 64000, "replay.n_subrings": 8})
    rp = HBMReplay(cfg, DEV)
    rp.fill_synthetic(episode_len=200, seed=3)
    B, H, Tn = 64, cfg.model.hidden, cfg.replay.seq_len + cfg.replay.n_step
    z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=DEV)   # noqa: E731
    g = torch.Generator(device=DEV).manual_seed(9)
    st, pb, rows = z(B, dt=torch.int32), z(B), z(Tn * B, dt=torch.int32)
    hs = [(rp.hs_cs, 0, z(B, H), z(B, H)), (rp.target_hs_cs, 5, z(B, H), z(B, H)),
          (rp.hs_cs, 5, z(B, H), z(B, H))]
    q = torch.zeros(4, dtype=torch.int32, device=DEV)
    idx = z(B, dt=torch.int32)
    res = {}

    def timed(name, fn):
        ts = []
        for _ in range(a.reps):
            rp.sample(B, idx, z(B))
            rp.priority.copy_(torch.rand(rp.capacity, generator=g, device=DEV) * 3)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        res[name + "_us"] = round(statistics.median(ts), 2)

    timed("tail", lambda: rp.prio_tail(idx, B, 40, 80, True))
    timed("sample", lambda: rp.sample_batch(B, st, pb, rows, Tn, hs, h_f32=True, qreset=q))
    timed("tail_then_sample", lambda: (rp.prio_tail(idx, B, 40, 80, True),
                                       rp.sample_batch(B, st, pb, rows, Tn, hs, h_f32=True, qreset=q)))
    timed("fused", lambda: rp.prio_tail_sample(idx, B, 40, 80, st, pb, rows, Tn, hs, True, q))
    timed("fused_skip2", lambda: rp.prio_tail_sample(idx, B, 40, 80, st, pb, rows, Tn, hs, True, q,
                                                     skip_xcds=2))
    res["dirty_last"] = int(rp.dirty_count.item())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
