"""R2D2 launcher (reference-compatible CLI: ``python main.py -n N``).

Parity target: ``/root/reference/main.py`` (``run()``: spawn 1 learner + N actors, Manager dict
for weights).  Modes:

  python main.py -n 4                          reference topology (learner + 4 actor processes,
                                               supervised, synthetic Atari env by default)
  python main.py --mode native --config pong --steps 2000
                                               MI355X-native: batched GPU actors + HIP learner
  python main.py --mode native --config pong --concurrent --steps 2000
                                               ... actors and learner running at the same time on
                                               disjoint CU sets of the GPU
  python main.py --mode native --config pong --cpu-actors 64 --steps 2000
                                               1 GPU learner + 64 CPU actor processes (shared-
                                               memory rings DMA'd into the HBM replay)
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 main.py --mode native --config seaquest8
                                               8-GPU data-parallel learner, actors on every GPU
  python main.py --mode inproc --config cartpole --steps 2000
                                               single process (CPU ok), CartPole plumbing config

Config overrides: ``--set learner.batch_size=16 replay.burn_in=20 ...``
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_r2d2_amd.config import get_config  # noqa: E402


def build_parser():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("-n", "--n_actors", type=int, default=1)
    p.add_argument("--mode", choices=["compat", "native", "inproc"], default="compat")
    p.add_argument("--config", default=None, help="preset: reference|cartpole|pong|atari57|seaquest8|dmlab30")
    p.add_argument("--steps", type=int, default=None, help="learner steps (default: run forever in compat)")
    p.add_argument("--env", default=None, help="override env name (synthetic|pong|cartpole)")
    p.add_argument("--device", default=None, help="learner device (compat/inproc)")
    p.add_argument("--actor-device", default="cpu", help="compat actors: cpu|cuda")
    p.add_argument("--metrics", default=None, help="JSONL metrics path")
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--capacity", type=int, default=None)
    p.add_argument("--set", nargs="*", default=[], help="dotted config overrides key=value")
    p.add_argument("--resume", default=None, help="full-state checkpoint to continue from (native)")
    p.add_argument("--cpu-actors", type=int, default=0,
                   help="native: N CPU actor processes feeding the GPU learner (instead of GPU actors)")
    p.add_argument("--concurrent", action="store_true",
                   help="native: GPU actor group and learner run simultaneously on disjoint CUs")
    p.add_argument("--actor-cus-per-xcd", type=int, default=0,
                   help="concurrent: CUs per XCD reserved for the actor group (0: share the chip)")
    p.add_argument("--actor-steps", type=int, default=1, help="native: env steps per learner step")
    p.add_argument("--actor-ranks", type=int, default=0,
                   help="native under torchrun: the last N ranks run GPU actor groups only and feed "
                        "the learner ranks (split topology, parallel/actor_ranks.py)")
    p.add_argument("--rounds", type=int, default=200, help="split topology: actor push rounds")
    return p


def run(argv=None):
    args = build_parser().parse_args(argv)
    preset = args.config or ("cartpole" if args.mode == "inproc" else
                             "pong" if args.mode == "native" else "reference")
    overrides = dict(kv.split("=", 1) for kv in args.set)
    if args.env:
        overrides["env.name"] = args.env
    cfg = get_config(preset, **overrides)
    if args.mode == "native" and args.actor_ranks > 0:
        from pytorch_r2d2_amd.runner import run_split
        out = run_split(cfg, rounds=args.rounds, actor_ranks=args.actor_ranks, capacity=args.capacity)
        out = {k: v for k, v in out.items() if k not in ("engine", "replay")}
    elif args.mode == "native" and args.cpu_actors > 0:
        from pytorch_r2d2_amd.runner import run_native_cpu_actors
        out = run_native_cpu_actors(cfg, args.cpu_actors, steps=args.steps or 1000,
                                    capacity=args.capacity, metrics_path=args.metrics)
        sup = out.pop("supervisor", None) or {}
        out["restarts"] = {k: v["restarts"] for k, v in sup.items() if v["restarts"]}
        out["exitcodes"] = {k: v["exitcodes"] for k, v in sup.items() if v["exitcodes"]}
    elif args.mode == "native":
        from pytorch_r2d2_amd.runner import run_native
        out = run_native(cfg, steps=args.steps or 1000, metrics_path=args.metrics,
                         checkpoint_dir=args.checkpoint_dir, capacity=args.capacity,
                         resume=args.resume, concurrent=args.concurrent,
                         actor_cus_per_xcd=args.actor_cus_per_xcd,
                         actor_steps_per_update=args.actor_steps)
        out.pop("driver", None)
    elif args.mode == "inproc":
        from pytorch_r2d2_amd.runner import run_inproc
        out = run_inproc(cfg, steps=args.steps or 1000, n_actors=args.n_actors,
                         device=args.device or "cpu", metrics_path=args.metrics)
        out.pop("learner", None)
    else:
        from pytorch_r2d2_amd.runner import run_compat
        out = run_compat(cfg, args.n_actors, steps=args.steps, actor_device=args.actor_device,
                         learner_device=args.device)
    print({k: v for k, v in out.items() if k not in ("losses", "returns")} if isinstance(out, dict) else out)
    return out


if __name__ == "__main__":
    run()
