"""Does the whole system learn -- and does the recurrent path learn what needs memory?

run_native (batched GPU actor + HIP learner, both HIP graphs) on the synthetic cue task
(envs/synthetic.py): the rewarded action changes every ``--switch`` agent steps and its column band
is painted bright on the frame.

* default: the cue is visible on every frame -- a reactive policy solves it (random policy =
  episode_len / A).
* ``--memory``: the cue is drawn ONLY on the first frame after a change (``env.cue_only_first``).
  A memoryless policy can score at most the ceiling (1/switch + (1 - 1/switch)/A) * episode_len
  (it sees the cue on one step in ``switch`` and guesses on the rest); the recurrent learner must
  carry the target in its LSTM state across the hidden steps.

Ablations (``--ablation``):
  zero_state   the learner ignores the stored recurrent state (zeros) and runs no burn-in:
               memory within a sequence only (what stored state + burn-in buy)
  memoryless   LSTM state reset before every actor step and learner sequences of one step from
               a zero state: no memory anywhere -- must stay at or below the ceiling

Prints one JSON line per run (mean return of successive windows of finished episodes).

    python tools/learn_check.py --steps 3000
    python tools/learn_check.py --memory --steps 6000
    python tools/learn_check.py --memory --ablation memoryless --steps 6000
"""
import argparse
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from pytorch_r2d2_amd.config import get_config  # noqa: E402
from pytorch_r2d2_amd.runner import run_native  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--episode-len", type=int, default=64)
    ap.add_argument("--switch", type=int, default=8)
    ap.add_argument("--memory", action="store_true", help="cue only on the first frame after a switch")
    ap.add_argument("--ablation", default="none", choices=("none", "zero_state", "memoryless"))
    ap.add_argument("--lr", type=float, default=2.5e-4)
    ap.add_argument("--optimizer", default="adam")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--burn-in", type=int, default=8)
    ap.add_argument("--learn", type=int, default=16)
    ap.add_argument("--dtype", default="fp32", help="fp32 | bf16 | both")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--concurrent", action="store_true")
    return ap.parse_args(argv)


def main():
    args = parse()
    for dt in (("bf16", "fp32") if args.dtype == "both" else (args.dtype,)):
        print(json.dumps(run_one(args, dt)), flush=True)


def memoryless_ceiling(episode_len: int, switch: int, n_actions: int) -> float:
    return (1.0 / switch + (1.0 - 1.0 / switch) / n_actions) * episode_len


def make_cfg(args, dtype):
    burn_in, learn, overlap = args.burn_in, args.learn, args.burn_in
    ov = {}
    if args.ablation == "zero_state":
        ov["learner.zero_stored_state"] = True
        # same sequence length, all of it learned from a zero state
        burn_in, learn, overlap = 0, args.burn_in + args.learn, args.burn_in
    elif args.ablation == "memoryless":
        ov["learner.zero_stored_state"] = True
        ov["actor.reset_state_every_step"] = True
        burn_in, learn, overlap = 0, 1, 1
    return get_config("atari57", **{
        "learner.compute_dtype": dtype, "seed": args.seed, "learner.batch_size": args.batch,
        "replay.burn_in": burn_in, "replay.learn": learn, "replay.overlap": overlap,
        "replay.n_step": 3, "actor.envs_per_actor": args.envs, "env.episode_len": args.episode_len,
        "env.switch": args.switch, "env.cue_only_first": bool(args.memory),
        "learner.initial_exploration": 4000, "learner.lr": args.lr,
        "learner.optimizer": args.optimizer, "learner.target_update_interval": 200,
        "learner.gamma": 0.9, **ov})


def run_one(args, dtype):
    cfg = make_cfg(args, dtype)
    t0 = time.time()
    out = run_native(cfg, steps=args.steps, log_every=max(1, args.steps // 10),
                     capacity=args.envs * 1000, concurrent=args.concurrent)
    rets = np.asarray(out["returns"], dtype=np.float64)
    w = max(1, len(rets) // 8)
    windows = [round(float(rets[i:i + w].mean()), 2) for i in range(0, len(rets) - w + 1, w)]
    A = cfg.model.n_actions
    ceil = memoryless_ceiling(args.episode_len, args.switch, A) if args.memory else None
    return {"metric": "synthetic_memory_task_return" if args.memory else "synthetic_cue_task_return",
            "dtype": dtype, "seed": args.seed, "ablation": args.ablation,
            "switch": args.switch, "cue_only_first": bool(args.memory),
            "seq": [cfg.replay.burn_in, cfg.replay.learn], "batch": cfg.learner.batch_size,
            "concurrent": bool(args.concurrent), "steps": args.steps, "episodes": int(len(rets)),
            "random_policy_return": args.episode_len / A, "memoryless_ceiling": ceil,
            "return_windows": windows, "final_window": windows[-1] if windows else None,
            "final_over_ceiling": (round(windows[-1] / ceil, 3) if ceil and windows else None),
            "first_loss": out["losses"][0], "last_loss": out["losses"][-1],
            "env_steps": out["env_steps"], "learner_steps_per_s": round(out["learner_steps_per_s"], 1),
            "wall_s": round(time.time() - t0, 1)}


if __name__ == "__main__":
    main()
