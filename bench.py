#!/usr/bin/env python3
"""Headline benchmark: R2D2 learner steps/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config atari57|reference|...]
                    [--dtype fp32|bf16] [--target-mode fixed|shifted|reference] [--profile-phases]

* Config (default ``atari57``): the R2D2 paper shapes -- batch 64 sequences of 80 steps
  (burn-in 40 + learning 40), n-step 5, value rescaling, IS weights, centered RMSprop -- on the
  reference network (``/root/reference/model.py``: 3-conv torso, LSTM 256, dueling head;
  2,037,095 parameters), synthetic uint8 frames in a 1M-row HBM replay, random-init weights.
  ``--config reference`` runs the reference's own shapes (B=8, T=20, n=3).
* Precision: ``--dtype`` defaults to the preset's ``learner.compute_dtype``.  ``fp32`` is the
  reference's precision (``/root/reference/model.py`` and ``learner.py`` run fp32): fp32 master
  weights, optimizer, activations, recurrent state and accumulation; every MFMA product is taken
  as three bf16 passes over hi/lo operand splits (``csrc/split.h``), whose error (~1e-5
  relative) is checked against an fp32 autograd oracle in ``tests/test_engine_gpu.py``.
* Formulation: ``--target-mode`` defaults to the preset.  ``fixed`` is the reference's 3-chain
  target (online on state, target on next_state, online on next_state with its own stored state
  and burn-in: ``/root/reference/learner.py:71-93`` with Q7 fixed); ``shifted`` is the R2D2
  paper's 2-chain form.
* A timed step is the FULL learner update: prioritized sample from the sum tree, torso on every
  frame of both nets, LSTM over every chain, head, TD loss, complete backward, (DP all-reduce),
  optimizer, weight repack, priority write-back + sum-tree repair.
* Multi-GPU (weak scaling): each rank runs the data-parallel learner on its own replay shard with
  the per-GPU batch fixed; one synchronous optimizer step per iteration over the global batch
  (64 x N sequences).  ``value`` is the WHOLE-JOB aggregate the driver's weak-scaling contract
  asks for: learner steps/s counted in the BASELINE's unit of work (one B=64 x 80-step batch
  trained), i.e. optimizer steps/s x N.  At N=1 it is exactly optimizer steps/s; at N>1 the JSON
  also carries ``optimizer_steps_per_sec`` (synchronous updates/s at global batch 64 x N) and
  ``sequences_per_sec`` so neither reading is hidden.
* Timing: W untimed warmup steps, then exactly K steps bracketed by barrier + synchronize on
  both sides; the max over ranks is reported by rank 0 as one JSON line.  The persistent
  kernels' error word is read after the timed loop: a non-zero word fails the run (exit 3).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINES = {
    "atari57": 5.0,      # R2D2 paper: ~5 learner updates/s at B=64 x 80 (1 GPU)
    "reference": 18.6,   # reference learner.py train() on 8-vCPU (measured in SURVEY §6)
}


def data_label(cfg) -> str:
    e = cfg.env
    c = e.channels_per_frame * e.n_stacks
    kind = "RGB" if e.channels_per_frame == 3 else "gray"
    return (f"synthetic {c}x{e.frame_h}x{e.frame_w} uint8 frames ({kind}, {e.n_stacks}-stack) "
            f"in HBM replay, random-init weights")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="atari57")
    ap.add_argument("--dtype", default="", choices=["", "fp32", "bf16"])
    ap.add_argument("--capacity", type=int, default=0)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--target-mode", default="")
    ap.add_argument("--profile-phases", action="store_true",
                    help="after the timed run, time each phase of 5 eager steps with HIP events "
                         "(+ roctx ranges) and add them to the JSON line under 'phases_ms'")
    ap.add_argument("--force-dp", action="store_true",
                    help="rehearsal under torchrun at ONE rank: the data-parallel step (segmented "
                         "graphs, RCCL all-reduces on the comm stream, CU reservation, shard-stats "
                         "all-gather) with one-rank collectives; labelled in 'parallelism'")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="config override, e.g. --set learner.lstm_xcd_pairs=0 (A/B experiments)")
    args = ap.parse_args(argv)

    import torch
    import torch.distributed as dist
    from pytorch_r2d2_amd.config import get_config
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
    from pytorch_r2d2_amd.utils.profiling import PhaseTimer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a box with fewer GPUs than ranks (R2D2_BENCH_SHARED=1):
    # ranks share GPUs round-robin and reduce over gloo (RCCL refuses two ranks on one GPU).
    # Never used for reported numbers: the JSON line says so in "parallelism".
    shared = os.environ.get("R2D2_BENCH_SHARED") == "1"
    if shared:
        local = local % torch.cuda.device_count()
    use_pg = world > 1 or args.force_dp
    if use_pg and "RANK" not in os.environ:   # --force-dp without a launcher: a one-rank group
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update({"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0",
                           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    if use_pg:
        torch.cuda.set_device(local)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    # one model seed for every rank (the engine also broadcasts rank 0's weights); the replay
    # contents differ per rank (their own shard)
    overrides = {"seed": 1234}
    if args.force_dp:
        overrides["dist.force_dp"] = True
    if args.target_mode:
        overrides["learner.target_mode"] = args.target_mode
    if args.dtype:
        overrides["learner.compute_dtype"] = args.dtype
    for kv in args.set:
        key, _, val = kv.partition("=")
        overrides[key] = val
    cfg = get_config(args.config, **overrides)
    cap = args.capacity or cfg.replay.capacity
    replay = HBMReplay(cfg, device, capacity=cap)
    replay.fill_synthetic(episode_len=400, seed=rank)
    eng = LearnerEngine(cfg, replay, device, rank=rank, world=world,
                        process_group=dist.group.WORLD if use_pg else None)
    use_graph = cfg.learner.use_graph and not args.no_graph
    if use_graph:
        eng.capture(warmup=2)
    # run_steps: the same steps as a step() loop; the hoisted graph mode replays runs of
    # learner.graph_chunk steps as one graph each (LearnerEngine.run_steps)
    eng.run_steps(args.warmup)
    if use_pg:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    eng.run_steps(args.steps)
    torch.cuda.synchronize(device)
    if use_pg:
        dist.barrier()
    dt = time.perf_counter() - t0
    err = eng.error_word()
    hoisted = None
    if getattr(eng, "hoist", False):   # target-net frames the last step's side launch computed
        n_tg = (eng.Tn - eng.t_lo_tg) * eng.B
        hoisted = [min(int(eng.tq[0].item()), n_tg), n_tg]
    if world > 1:
        tt = torch.tensor([dt, float(err)], device=device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt, err = float(tt[0].item()), int(tt[1].item())
    ms = dt / args.steps * 1e3
    opt_steps = args.steps / dt
    loss = eng.loss_value()
    phases = None
    if args.profile_phases:
        timer = PhaseTimer()
        for _ in range(5):
            eng.step_eager(timer=timer)
        phases = {k: round(v, 4) for k, v in timer.summary().items()}
        err = max(err, eng.error_word())
    rc, lc = cfg.replay, cfg.learner
    base = BASELINES.get(args.config)
    if rank == 0:
        out = {
            "metric": "learner_steps_per_sec",
            "value": round(opt_steps * world, 3),
            "unit": ("learner steps/s of the whole job, one step = a %d x %d-step sequence batch "
                     "(= optimizer steps/s x %d ranks; global batch %d)"
                     % (lc.batch_size, rc.seq_len, world, lc.batch_size * world)),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(opt_steps * world / base, 3) if base else None,
            "dtype": lc.compute_dtype,
            "data": data_label(cfg),
            "config": {
                "model": "r2d2-qnet (reference model.py: conv32x3 + LSTM%d + dueling, %d actions)"
                         % (cfg.model.hidden, cfg.model.n_actions),
                "preset": cfg.name,
                "global_batch": lc.batch_size * world,
                "per_gpu_batch": lc.batch_size,
                "seq_len": rc.seq_len,
                "burn_in": rc.burn_in,
                "n_step": rc.n_step,
                "target_mode": lc.target_mode,
                "matmul": ("bf16x3 split (fp32 accumulate, fp32 state/storage)"
                           if lc.compute_dtype == "fp32" else "bf16 operands, fp32 accumulate"),
                "replay_rows_per_gpu": replay.capacity,
                "parallelism": "dp%d" % world + ("-shared-gpu-gloo-rehearsal" if shared else "")
                               + ("-forced-dp-rehearsal" if args.force_dp and world == 1 else ""),
                "hip_graph": bool(use_graph),
                # step k's priority tail, step k+1's sample and part of its target-net torso
                # run on a side stream beside step k's BPTT (learner.hoist; bit-identical)
                "hoisted_step": bool(getattr(eng, "hoist", False)),
                # consecutive hoisted steps replayed per graph (1 = one graph per step)
                "graph_chunk": eng._chunk_len() if use_graph else 0,
                "dp_graph": eng.dp_graph_label(),
            },
            "optimizer_steps_per_sec": round(opt_steps, 3),
            "sequences_per_sec": round(opt_steps * lc.batch_size * world, 1),
            "per_gpu_sequences_per_sec": round(opt_steps * lc.batch_size, 1),
            "final_loss": loss,
            "kernel_error_word": err,
        }
        if phases is not None:
            out["phases_ms"] = phases
        if hoisted is not None:
            out["hoisted_target_frames"] = hoisted
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.destroy_process_group()
    if err:
        print(f"bench: persistent-kernel error word {err:#x} (hand-off spin timed out)",
              file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
