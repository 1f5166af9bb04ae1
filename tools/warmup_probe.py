"""Per-step device time of the first steps after capture (bench.py's setup, atari57 paper config):
events around each graph replay, so a slow start (first replays of each graph, clock ramp, cold
caches / TLBs) shows up step by step.  Prints one JSON line.

    python tools/warmup_probe.py [--steps 60] [--set KEY=VALUE ...]
"""
import argparse
import json
import time

import torch

from pytorch_r2d2_amd.config import get_config
from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--capacity", type=int, default=0)
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--spin-ms", type=float, default=0.0, help="busy-wait on the host before stepping")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    over = {"seed": 1234}
    for kv in a.set:
        k, _, v = kv.partition("=")
        over[k] = v
    cfg = get_config("atari57", **over)
    rp = HBMReplay(cfg, dev, capacity=a.capacity or cfg.replay.capacity)
    rp.fill_synthetic(episode_len=400, seed=0)
    eng = LearnerEngine(cfg, rp, dev)
    t0 = time.perf_counter()
    eng.capture(warmup=2)
    torch.cuda.synchronize()
    t_cap = time.perf_counter() - t0
    if a.spin_ms:
        time.sleep(a.spin_ms / 1e3)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    ev[0].record()
    for i in range(a.steps):
        eng.step()
        ev[i + 1].record()
    torch.cuda.synchronize()
    us = [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(a.steps)]
    print(json.dumps({"capture_s": round(t_cap, 2), "step_us": us,
                      "first20_mean_us": round(sum(us[5:25]) / 20, 1),
                      "last20_mean_us": round(sum(us[-20:]) / 20, 1), "err": eng.error_word()}))


if __name__ == "__main__":
    main()
