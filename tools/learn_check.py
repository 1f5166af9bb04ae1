"""Does the whole system learn?  run_native (batched GPU actor + HIP learner, both HIP graphs)
on the synthetic cue task: the frame shows a bright column band for the rewarded action
(reward 1 when the action matches, target switches every 8 steps), so a random policy scores
episode_len / n_actions and a learned one close to episode_len.  Prints the mean return of
successive windows of finished episodes as one JSON line.

    python tools/learn_check.py --steps 3000
    python tools/learn_check.py --steps 3000 --dtype both     # bf16 vs fp32 (split) learning parity
"""
import argparse
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from pytorch_r2d2_amd.config import get_config  # noqa: E402
from pytorch_r2d2_amd.runner import run_native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--episode-len", type=int, default=64)
    ap.add_argument("--lr", type=float, default=2.5e-4)
    ap.add_argument("--optimizer", default="adam")
    ap.add_argument("--dtype", default="fp32", help="fp32 | bf16 | both")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--concurrent", action="store_true")
    args = ap.parse_args()
    for dt in (("bf16", "fp32") if args.dtype == "both" else (args.dtype,)):
        run_one(args, dt)


def run_one(args, dtype):
    cfg = get_config("atari57", **{"learner.compute_dtype": dtype, "seed": args.seed,
        "learner.batch_size": 32, "replay.burn_in": 8, "replay.learn": 16, "replay.overlap": 8,
        "replay.n_step": 3, "actor.envs_per_actor": args.envs, "env.episode_len": args.episode_len,
        "learner.initial_exploration": 4000, "learner.lr": args.lr,
        "learner.optimizer": args.optimizer, "learner.target_update_interval": 200,
        "learner.gamma": 0.9})
    t0 = time.time()
    out = run_native(cfg, steps=args.steps, log_every=max(1, args.steps // 10),
                     capacity=args.envs * 1000, concurrent=args.concurrent)
    rets = np.asarray(out["returns"], dtype=np.float64)
    w = max(1, len(rets) // 8)
    windows = [round(float(rets[i:i + w].mean()), 2) for i in range(0, len(rets) - w + 1, w)]
    res = {"metric": "synthetic_cue_task_return", "dtype": dtype, "seed": args.seed,
           "concurrent": bool(args.concurrent), "steps": args.steps, "episodes": int(len(rets)),
           "random_policy_return": args.episode_len / cfg.model.n_actions,
           "return_windows": windows, "first_loss": out["losses"][0], "last_loss": out["losses"][-1],
           "env_steps": out["env_steps"], "wall_s": round(time.time() - t0, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
