"""Actor + learner throughput of the native single-GPU topology: serial (the actor group and the
learner alternate on one stream) vs concurrent (engine/concurrent.py: disjoint CU sets, event
pipelined).  Prints one JSON line per mode.

    python tools/bench_native.py --preset atari57 --steps 300 --actor-steps 1 --modes serial,concurrent
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_r2d2_amd.config import get_config  # noqa: E402
from pytorch_r2d2_amd.runner import run_native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="atari57")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--actor-steps", type=int, default=1)
    ap.add_argument("--envs", type=int, default=None)
    ap.add_argument("--capacity", type=int, default=None)
    ap.add_argument("--actor-cus-per-xcd", type=int, default=0)
    ap.add_argument("--learner-priority", type=int, default=0)
    ap.add_argument("--modes", default="serial,concurrent")
    ap.add_argument("--set", nargs="*", default=[])
    a = ap.parse_args()
    over = dict(kv.split("=", 1) for kv in a.set)
    if a.envs:
        over["actor.envs_per_actor"] = a.envs
    cfg = get_config(a.preset, **over)
    E = cfg.actor.envs_per_actor
    cap = a.capacity or E * 4096
    warm = E * (cfg.replay.seq_len + cfg.replay.n_step + 2 * cfg.replay.overlap)
    for mode in a.modes.split(","):
        out = run_native(cfg, steps=a.steps, actor_steps_per_update=a.actor_steps, warmup_rows=warm,
                         capacity=cap, log_every=10 ** 9, concurrent=(mode == "concurrent"),
                         actor_cus_per_xcd=a.actor_cus_per_xcd, learner_priority=a.learner_priority,
                         check_every=100)
        rec = {"mode": mode, "preset": a.preset, "envs": E, "actor_steps_per_learner_step": a.actor_steps,
               "actor_cus_per_xcd": a.actor_cus_per_xcd, "learner_priority": a.learner_priority,
               "learner_steps_per_s": round(out["learner_steps_per_s"], 1),
               "env_steps_per_s": round(out["env_steps_per_s"], 1),
               "learner_cus": out["learner_cus"], "dtype": cfg.learner.compute_dtype,
               "batch": cfg.learner.batch_size, "seq_len": cfg.replay.seq_len}
        print(json.dumps(rec), flush=True)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
