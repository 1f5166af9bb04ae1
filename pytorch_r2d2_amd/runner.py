"""Training entry points.

``run_native``  -- MI355X-native topology: one process per GPU (torchrun, RCCL); on every rank a
                   ``BatchedActor`` group (E vectorised envs, one HBM sub-ring each) feeds the
                   rank's HBM replay shard and a data-parallel ``LearnerEngine`` trains on it
                   (bucketed all-reduce overlapped with the conv backward).  Weights reach the
                   co-located actors zero-copy; nothing but gradients crosses xGMI.
``run_compat``  -- the reference topology (main.py:10-33): a learner process + N single-env
                   actor processes, Manager-dict weights, file transport (fixed, tensor-only),
                   under the ``Supervisor`` (restarts crashed actors).
``run_inproc``  -- single process, CPU or GPU, host replay + torch learner + single-env actors
                   stepping inline (the CartPole plumbing config, tests).
"""
from __future__ import annotations

import os
import time
from typing import Dict, Optional

import numpy as np
import torch

from .config import R2D2Config


def run_native(cfg: R2D2Config, steps: int = 1000, actor_steps_per_update: int = 1,
               warmup_rows: Optional[int] = None, metrics_path: Optional[str] = None,
               checkpoint_dir: Optional[str] = None, log_every: int = 100, use_graph: bool = True,
               capacity: Optional[int] = None, resume: Optional[str] = None) -> Dict:
    from .actor_batched import BatchedActor, engine_weights
    from .engine.learner_engine import LearnerEngine
    from .engine.replay_hbm import HBMReplay
    from .envs.synthetic import VecSyntheticAtari
    from .parallel.dist import init_distributed
    from .utils.checkpoint import save_full_checkpoint, save_reference_checkpoint
    from .utils.metrics import MetricsLogger

    info = init_distributed()
    dev = info.device
    E = cfg.actor.envs_per_actor
    torch.manual_seed(cfg.seed)
    replay = HBMReplay(cfg, dev, capacity=capacity or cfg.replay.capacity, n_subrings=E)
    import torch.distributed as dist
    eng = LearnerEngine(cfg, replay, dev, rank=info.rank, world=info.world,
                        process_group=dist.group.WORLD if info.world > 1 else None)
    env = VecSyntheticAtari(E, dev, seed=cfg.seed + 101 * info.rank, episode_len=cfg.env.episode_len,
                            n_actions=cfg.model.n_actions,
                            n_stacks=cfg.env.channels_per_frame * cfg.env.n_stacks,
                            shape=(cfg.env.frame_h, cfg.env.frame_w))
    start = 0
    if resume:
        from .utils.checkpoint import load_full_checkpoint, restore_rng
        obj = load_full_checkpoint(resume)
        restore_rng(obj)
        eng.load_full_state(obj)
        start = int(obj["step"])
    on, tg = engine_weights(eng)
    actor = BatchedActor(cfg, replay, env, on, tg, global_env_offset=info.rank * E,
                         total_envs=info.world * E, seed=cfg.seed + info.rank)
    mlog = MetricsLogger(metrics_path, rank=info.rank) if metrics_path else None
    warm = warmup_rows if warmup_rows is not None else min(cfg.learner.initial_exploration,
                                                           replay.capacity // 2)
    t0 = time.perf_counter()
    while replay.total_written < warm or int(replay.n_valid.item()) < cfg.learner.batch_size:
        actor.step()
    if info.world > 1:
        dist.barrier()
    t_warm = time.perf_counter() - t0
    if use_graph and cfg.learner.use_graph:
        eng.capture(warmup=1)
    if use_graph and cfg.actor.use_graph and actor.can_capture:
        actor.capture(warmup=1)
    losses = []
    t1 = time.perf_counter()
    for it in range(steps):
        for _ in range(actor_steps_per_update):
            actor.step()
        eng.step()
        if (it + 1) % log_every == 0 or it == steps - 1:
            loss = eng.loss_value()
            losses.append(loss)
            rets = actor.finished_returns[-64:]
            rec = dict(step=it + 1, loss=loss, replay_rows=replay.size,
                       n_valid=int(replay.n_valid.item()), env_steps=actor.env_steps,
                       mean_return=float(np.mean(rets)) if rets else None,
                       learner_steps_per_s=(it + 1) / (time.perf_counter() - t1))
            if mlog:
                mlog.log("native", **rec)
            if info.is_main:
                print("[native]", rec, flush=True)
        if checkpoint_dir and info.is_main and (start + it + 1) % cfg.learner.checkpoint_interval == 0:
            save_reference_checkpoint(eng.state_dict(), start + it + 1, checkpoint_dir)
    torch.cuda.synchronize(dev)
    eng.check_errors()
    out = {"steps": steps, "warmup_s": t_warm, "train_s": time.perf_counter() - t1,
           "losses": losses, "returns": list(actor.finished_returns), "env_steps": actor.env_steps}
    if checkpoint_dir and info.is_main:
        save_full_checkpoint(os.path.join(checkpoint_dir, "full_last.pt"), eng.state_dict(),
                             eng.target_state_dict(), None, start + steps, cfg, eng.full_state_extra())
    return out


def run_inproc(cfg: R2D2Config, steps: int = 1000, n_actors: int = 1, device: str = "cpu",
               actor_steps_per_update: int = 4, log_every: int = 100,
               metrics_path: Optional[str] = None, seed: int = 0) -> Dict:
    """Single process: host replay, torch learner, single-env actors stepping inline."""
    from .actor import Actor
    from .learner import Learner

    shared = {}
    learner = Learner(n_actors, shared, device=device, cfg=cfg, backend="torch",
                      metrics_path=metrics_path)
    actors = [Actor(i, n_actors, shared, device=device, cfg=cfg, seed=seed) for i in range(n_actors)]
    # actors write straight into the learner's host replay (no files in-process)
    for a in actors:
        a.replay_memory = learner.replay_memory
        a.memory_save_interval = 1 << 30
        a.episode_start_index = learner.replay_memory.index
    losses, t0 = [], time.perf_counter()
    it = 0
    while it < steps:
        for a in actors:
            for _ in range(actor_steps_per_update):
                a.step()
        if learner.replay_size() > learner.initial_exploration and \
                int(learner.replay_memory.memory["is_seq_start"].sum()) > 0:
            loss = learner.train()
            learner.n_epochs += 1
            learner.interval()
            it += 1
            if it % log_every == 0:
                losses.append(loss)
                rets = [r for a in actors for r in a.episode_returns[-10:]]
                print(f"[inproc] step {it} loss {loss:.4f} mean_return "
                      f"{np.mean(rets) if rets else float('nan'):.1f}", flush=True)
            if it % cfg.actor.net_load_interval == 0:
                for a in actors:
                    a.load_model()
    return {"losses": losses, "returns": [r for a in actors for r in a.episode_returns],
            "time_s": time.perf_counter() - t0, "learner": learner}


def run_compat(cfg: R2D2Config, n_actors: int, steps: Optional[int] = None,
               actor_device: str = "cpu", learner_device: Optional[str] = None,
               memory_path: Optional[str] = None, timeout_s: Optional[float] = None,
               stall_timeout_s: float = 0.0) -> Dict:
    """Reference process topology under the supervisor."""
    import multiprocessing as mp

    from .actor import actor_process
    from .learner import learner_process
    from .utils.supervisor import RoleSpec, Supervisor

    ctx = mp.get_context("spawn")
    manager = ctx.Manager()
    shared = manager.dict()
    memory_path = memory_path or os.path.join(".", "logs", "memory")
    roles = [RoleSpec("learner", learner_process, (n_actors, shared),
                      dict(device=learner_device, cfg=cfg, max_steps=steps, memory_path=memory_path),
                      restartable=False)]
    for i in range(n_actors):
        dev = actor_device
        if actor_device == "cuda" and torch.cuda.is_available():
            dev = f"cuda:{(i % max(1, torch.cuda.device_count() - 1)) + (1 if torch.cuda.device_count() > 1 else 0)}"
        roles.append(RoleSpec(f"actor{i}", actor_process, (i, n_actors, shared, dev),
                              dict(cfg=cfg, memory_path=memory_path),
                              stall_timeout_s=stall_timeout_s))
    sup = Supervisor(roles)

    def learner_done():
        p = sup.procs[0]
        return p is None or (not p.is_alive() and p.exitcode == 0)

    report = sup.run(until=learner_done, timeout_s=timeout_s)
    manager.shutdown()
    return report
