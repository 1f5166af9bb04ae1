"""Actor-side throughput: env steps/s of one BatchedActor group (E synthetic Atari envs, both
nets' torso + LSTM step + dueling head per env step, device-side n-step / priorities / replay
writes), and the interleaved actor+learner loop of runner.run_native.

    python tools/bench_actor.py --config atari57 --envs 64,256 --steps 200
Prints one JSON line.  The R2D2 paper's CPU actors run ~260 env steps/s each."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from pytorch_r2d2_amd.actor_batched import BatchedActor, engine_weights  # noqa: E402
from pytorch_r2d2_amd.config import get_config  # noqa: E402
from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine  # noqa: E402
from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay  # noqa: E402
from pytorch_r2d2_amd.envs.synthetic import VecSyntheticAtari  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="atari57")
    ap.add_argument("--envs", default="64,256")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--capacity", type=int, default=1 << 18)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-loop", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {"metric": "actor_env_steps_per_sec", "config": args.config}
    for E in [int(v) for v in args.envs.split(",")]:
        cfg = get_config(args.config, **{"actor.envs_per_actor": E})
        cap = (args.capacity // E) * E
        replay = HBMReplay(cfg, dev, capacity=cap, n_subrings=E)
        eng = LearnerEngine(cfg, replay, dev)
        env = VecSyntheticAtari(E, dev, seed=1, episode_len=cfg.env.episode_len,
                                n_actions=cfg.model.n_actions,
                                n_stacks=cfg.env.channels_per_frame * cfg.env.n_stacks,
                                shape=(cfg.env.frame_h, cfg.env.frame_w))
        on, tg = engine_weights(eng)
        actor = BatchedActor(cfg, replay, env, on, tg, seed=3)
        for _ in range(args.warmup):
            actor.step()
        if not args.no_graph and actor.can_capture:
            actor.capture(warmup=1)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            actor.step()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        out[f"E{E}_env_steps_per_s"] = round(args.steps * E / dt, 1)
        out[f"E{E}_ms_per_actor_step"] = round(dt / args.steps * 1e3, 3)
        # interleaved loop (run_native): one actor step + one learner step
        if args.no_loop:
            continue
        while int(replay.n_valid.item()) < cfg.learner.batch_size:
            actor.step()
        if cfg.learner.use_graph:
            eng.capture(warmup=1)
        for _ in range(5):
            actor.step()
            eng.step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        n = max(20, args.steps // 4)
        for _ in range(n):
            actor.step()
            eng.step()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        out[f"E{E}_loop_ms_per_iter"] = round(dt / n * 1e3, 3)
        del actor, eng, replay, env
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
