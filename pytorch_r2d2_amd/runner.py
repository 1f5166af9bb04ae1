"""Training entry points.

``run_native``  -- MI355X-native topology: one process per GPU (torchrun, RCCL); on every rank a
                   ``BatchedActor`` group (E vectorised envs, one HBM sub-ring each) feeds the
                   rank's HBM replay shard and a data-parallel ``LearnerEngine`` trains on it
                   (bucketed all-reduce overlapped with the conv backward).  Weights reach the
                   co-located actors zero-copy; nothing but gradients crosses xGMI.
``run_compat``  -- the reference topology (main.py:10-33): a learner process + N single-env
                   actor processes, Manager-dict weights, file transport (fixed, tensor-only),
                   under the ``Supervisor`` (restarts crashed actors).
``run_split``   -- learner ranks + actor-only ranks: device-packed trajectory records over RCCL
                   send/recv, weights broadcast from learner rank 0 (parallel/actor_ranks.py).
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
               capacity: Optional[int] = None, resume: Optional[str] = None,
               concurrent: bool = False, actor_cus_per_xcd: int = 0, learner_priority: int = 0,
               beat=None,
               check_every: int = 200, on_step=None) -> Dict:
    """``concurrent``: actor group and learner run simultaneously on disjoint CU sets
    (engine/concurrent.py; ``actor_steps_per_update`` env steps per learner step), else they
    alternate on one stream.  ``beat``: supervisor heartbeat; the persistent kernels' error word
    is checked every ``check_every`` steps (a hand-off timeout stops the run with an error)."""
    from .actor_batched import BatchedActor, engine_weights
    from .engine.learner_engine import LearnerEngine
    from .engine.replay_hbm import HBMReplay
    from .envs.synthetic import VecSyntheticAtari
    from .parallel.dist import init_distributed
    from .utils.checkpoint import save_full_checkpoint, save_reference_checkpoint
    from .utils.faults import Liveness
    from .utils.metrics import MetricsLogger

    info = init_distributed()
    dev = info.device
    E = cfg.actor.envs_per_actor
    torch.manual_seed(cfg.seed)
    s_act = s_learn = None
    n_cus_learner = xcd_cus = None
    n_cus_actor = 256
    if concurrent and dev.type == "cuda" and actor_cus_per_xcd > 0:
        from .parallel.placement import split_chip
        s_act, s_learn, n_cus_actor, n_cus_learner, xcd_cus = split_chip(dev, actor_cus_per_xcd)
    replay = HBMReplay(cfg, dev, capacity=capacity or cfg.replay.capacity, n_subrings=E)
    import torch.distributed as dist
    eng = LearnerEngine(cfg, replay, dev, rank=info.rank, world=info.world,
                        process_group=dist.group.WORLD if info.world > 1 else None,
                        n_cus=n_cus_learner, xcd_cus=xcd_cus)
    env = VecSyntheticAtari(E, dev, seed=cfg.seed + 101 * info.rank, episode_len=cfg.env.episode_len,
                            n_actions=cfg.model.n_actions,
                            n_stacks=cfg.env.channels_per_frame * cfg.env.n_stacks,
                            shape=(cfg.env.frame_h, cfg.env.frame_w), switch=cfg.env.switch,
                            cue_only_first=cfg.env.cue_only_first)
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
    if concurrent:
        # the actor group's kernels must never need co-residency on the learner's CUs
        actor.lstm_step = True
    mlog = MetricsLogger(metrics_path, rank=info.rank) if metrics_path else None
    live = Liveness("learner", info.rank, beat)
    warm = warmup_rows if warmup_rows is not None else min(cfg.learner.initial_exploration,
                                                           replay.capacity // 2)
    t0 = time.perf_counter()
    while replay.total_written < warm or int(replay.n_valid.item()) < cfg.learner.batch_size:
        actor.step()
        live.tick(0)
    if info.world > 1:
        dist.barrier()
    t_warm = time.perf_counter() - t0
    if use_graph and cfg.learner.use_graph:
        eng.capture(warmup=1)
    drv = None
    if concurrent:
        from .engine.concurrent import ConcurrentDriver
        actor.n_workers = n_cus_actor
        drv = ConcurrentDriver(eng, actor, steps_per_round=actor_steps_per_update,
                               actor_stream=s_act.stream if s_act else None,
                               learner_stream=s_learn.stream if s_learn else None,
                               capture=use_graph and cfg.actor.use_graph and actor.can_capture,
                               learner_priority=learner_priority)
        if on_step is not None:
            drv.on_learner_step = on_step
    elif use_graph and cfg.actor.use_graph and actor.can_capture:
        actor.capture(warmup=1)
    losses = []
    env0 = actor.env_steps
    t1 = time.perf_counter()
    for it in range(steps):
        live.tick(start + it)
        if drv is not None:
            drv.round()
        else:
            for _ in range(actor_steps_per_update):
                actor.step()
            eng.step()
            if on_step is not None:
                on_step(it)
        if check_every and (it + 1) % check_every == 0:
            eng.check_errors()
        if (it + 1) % log_every == 0 or it == steps - 1:
            if drv is not None:
                torch.cuda.current_stream(dev).wait_stream(drv.s_learn)
            st = eng.diagnostics()
            loss = st["loss"]
            losses.append(loss)
            rets = actor.finished_returns[-64:]
            el = time.perf_counter() - t1
            rec = dict(step=it + 1, replay_rows=replay.size, env_steps=actor.env_steps,
                       mean_return=float(np.mean(rets)) if rets else None,
                       return_by_eps=actor.returns_by_epsilon(),
                       learner_steps_per_s=(it + 1) / el, dp_imbalance=eng.dp_imbalance(),
                       env_steps_per_s=(actor.env_steps - env0) / el, **st)
            if mlog:
                mlog.log("native", **rec)
            if info.is_main:
                print("[native]", rec, flush=True)
        # the learner step counter is the engine's (it also counts the capture warm-up steps,
        # which really trained), so checkpoint names / resume agree with the device step
        if checkpoint_dir and info.is_main and eng.steps_done % cfg.learner.checkpoint_interval == 0:
            if drv is not None:
                torch.cuda.current_stream(dev).wait_stream(drv.s_learn)
            save_reference_checkpoint(eng.state_dict(), eng.steps_done, checkpoint_dir)
    if drv is not None:
        drv.finish()
        drv.check_errors()
    torch.cuda.synchronize(dev)
    train_s = time.perf_counter() - t1
    eng.check_errors()
    out = {"steps": steps, "warmup_s": t_warm, "train_s": train_s,
           "learner_steps_per_s": steps / train_s,
           "env_steps_per_s": (actor.env_steps - env0) / train_s,
           "losses": losses, "returns": list(actor.finished_returns), "env_steps": actor.env_steps,
           "concurrent": bool(concurrent), "learner_cus": eng.n_cus,
           "weights_version": drv.version if drv is not None else None}
    if checkpoint_dir and info.is_main:
        save_full_checkpoint(os.path.join(checkpoint_dir, "full_last.pt"), eng.state_dict(),
                             eng.target_state_dict(), None, eng.steps_done, cfg, eng.full_state_extra())
    if drv is not None:
        out["driver"] = drv
    for s_ in (s_act, s_learn):
        if s_ is not None:
            s_.close()
    return out


def run_split(cfg: R2D2Config, rounds: int = 200, actor_ranks: Optional[int] = None,
              capacity: Optional[int] = None, log_every: int = 50, use_graph: bool = True,
              backend: str = "auto", learner_steps: Optional[int] = None,
              actor_delay_s: float = 0.0) -> Dict:
    """Split topology (parallel/actor_ranks.py): learner ranks 0 .. L-1 (data parallel), actor
    ranks L .. W-1 (``BatchedActor`` groups only), decoupled like the reference's processes:

    * every actor rank runs ``rounds`` rounds of ``dist.push_rows`` env steps and pushes one
      record per round over its asynchronous link (blocking only when all ``dist.push_slots``
      records are untaken), taking weight snapshots between rounds;
    * every learner rank polls its links between steps and ingests what has arrived; once every
      learner shard holds a batch of sequences the learners train ``learner_steps`` steps
      (default ``rounds * dist.learner_steps_per_round``) without waiting on any actor, learner
      0 publishing weights every ``dist.publish_steps`` steps; then they drain the remaining
      records and close the weight links.

    ``actor_delay_s``: extra host time per round on actor rank W-1 (a slow actor, tests)."""
    import torch.distributed as dist

    from .actor_batched import BatchedActor, PackedWeights
    from .engine.layout import ParamLayout
    from .engine.learner_engine import LearnerEngine
    from .engine.replay_hbm import HBMReplay
    from .envs.synthetic import VecSyntheticAtari
    from .parallel.actor_ranks import TrajectoryPusher, TrajectoryReceiver, WeightLinks, split_roles
    from .parallel.dist import init_distributed
    from .utils.faults import Liveness

    info = init_distributed(backend=backend)
    dev = info.device
    A = int(actor_ranks if actor_ranks is not None else cfg.dist.actor_ranks)
    learners, actors, feeds = split_roles(info.world, A)
    dc, rc = cfg.dist, cfg.replay
    E, K = cfg.actor.envs_per_actor, int(dc.push_rows)
    W = rc.seq_len + rc.n_step
    # every rank creates the same groups in the same order
    g_learn = dist.new_group(learners) if len(learners) > 1 else None
    # weight snapshots (learner 0 -> actor ranks) on a group of their own: over RCCL a group's
    # point-to-point traffic between two ranks shares one communicator and stream, so with the
    # records (actor -> learner) on the same group a weight send queued on learner 0 ahead of a
    # record recv, and a record send queued on the actor ahead of the weight recv, could each
    # wait (payloads larger than the per-peer buffer) for the recv stuck behind the other
    g_w = dist.new_group(sorted(set([learners[0]] + actors)))
    torch.manual_seed(cfg.seed)
    L = ParamLayout(cfg.model, cfg.env)
    live = Liveness("learner" if info.rank in learners else "actor", info.rank, None)
    out = {"rank": info.rank, "role": "learner" if info.rank in learners else "actor",
           "rounds": rounds, "world": info.world, "actor_ranks": A}
    P = max(1, int(dc.publish_steps))
    if learner_steps is None:
        learner_steps = rounds * int(dc.learner_steps_per_round)
    if info.rank in learners:
        mine = [a for a in actors if feeds[a] == info.rank]
        n_sub = max(1, E * len(mine))
        cap = capacity or cfg.replay.capacity
        replay = HBMReplay(cfg, dev, capacity=max(cap // n_sub, 2 * (K + W)) * n_sub, n_subrings=n_sub)
        eng = LearnerEngine(cfg, replay, dev, rank=learners.index(info.rank), world=len(learners),
                            process_group=g_learn)
        recv = TrajectoryReceiver(replay, mine, E, K)
        wl = (WeightLinks(L.padded, dev, actors, learners[0], "learner", group=g_w)
              if info.rank == learners[0] else None)
        PS = max(1, int(dc.poll_steps))
        if wl is not None:
            wl.publish(eng.master, eng.target)
        steps, polls, t_train, captured = 0, 0, None, False
        warm = torch.zeros(1, dtype=torch.float32, device=dev)
        t0 = time.perf_counter()
        while steps < learner_steps:
            live.tick(steps)
            if captured and steps % PS:       # rate-limited store round trips while training
                got = 0
            else:
                polls += 1
                got = recv.poll()
            if not captured:
                # every learner shard must hold a batch of sequences before any of them steps
                # (the DP step's collectives need all learner ranks in it)
                warm.fill_(float(replay.n_valid.item() >= cfg.learner.batch_size))
                if g_learn is not None:
                    dist.all_reduce(warm, op=dist.ReduceOp.MIN, group=g_learn)
                if warm.item() > 0:
                    if use_graph and cfg.learner.use_graph:
                        eng.capture(warmup=1)
                    captured = True
                    torch.cuda.synchronize(dev)
                    t_train = time.perf_counter()
                elif not got:
                    time.sleep(0.0005)
                continue
            eng.step()
            steps += 1
            if wl is not None and steps % P == 0:
                wl.publish(eng.master, eng.target)
            if info.rank == learners[0] and log_every and steps % log_every == 0:
                print(f"[split] learner steps {steps} loss {eng.loss_value():.4f} rows {recv.rows}",
                      flush=True)
        torch.cuda.synchronize(dev)
        t_end = time.perf_counter()
        recv.drain(rounds)
        if wl is not None:
            wl.close()
        torch.cuda.synchronize(dev)
        eng.check_errors()
        el = t_end - t_train if t_train else 0.0
        out.update(learner_steps=steps, learner_steps_per_s=steps / el if el > 0 else 0.0,
                   rows_ingested=recv.rows, records=recv.records,
                   weights_version=wl.published if wl is not None else None,
                   n_valid=int(replay.n_valid.item()), final_loss=eng.loss_value() if steps else None,
                   ingest_err=int(replay.ingest_err.item()), warm_s=(t_train or t_end) - t0,
                   engine=eng, replay=replay)
    else:
        cap_e = max(2 * (K + W + rc.n_step), 512)
        replay = HBMReplay(cfg, dev, capacity=cap_e * E, n_subrings=E)
        w_on, w_tg = PackedWeights(L, dev), PackedWeights(L, dev)
        wl = WeightLinks(L.padded, dev, actors, learners[0], "actor", group=g_w)
        wl.attach(w_on, w_tg)
        while wl.taken == 0:          # the initial snapshot
            if wl.poll() == 0:
                time.sleep(0.0005)
        env = VecSyntheticAtari(E, dev, seed=cfg.seed + 101 * info.rank, episode_len=cfg.env.episode_len,
                                n_actions=cfg.model.n_actions,
                                n_stacks=cfg.env.channels_per_frame * cfg.env.n_stacks,
                                shape=(cfg.env.frame_h, cfg.env.frame_w), switch=cfg.env.switch,
                                cue_only_first=cfg.env.cue_only_first)
        idx = actors.index(info.rank)
        actor = BatchedActor(cfg, replay, env, w_on, w_tg, global_env_offset=idx * E,
                             total_envs=A * E, seed=cfg.seed + info.rank)
        # an RCCL send may sit on this chip while the actor keeps stepping: the actor group's
        # kernels must never need co-residency of the whole grid
        actor.lstm_step = True
        if use_graph and cfg.actor.use_graph and actor.can_capture:
            actor.capture(warmup=0)
        push = TrajectoryPusher(replay, K, feeds[info.rank], slots=int(dc.push_slots))
        slow = actor_delay_s if info.rank == actors[-1] else 0.0
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for r in range(rounds):
            live.tick(r)
            for _ in range(K):
                actor.step()
            if slow:
                torch.cuda.synchronize(dev)
                time.sleep(slow)
            push.push(r)
            wl.poll()
        push.finish()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        wl.wait_closed()
        out.update(env_steps=actor.env_steps, env_steps_per_s=actor.env_steps / el,
                   windows=push.windows, weights_version=wl.taken, push_stalls=push.link.stalls,
                   push_stall_s=push.link.stall_s, returns=list(actor.finished_returns))
    return out


def run_native_cpu_actors(cfg: R2D2Config, n_actors: int, steps: int = 1000,
                          actor_max_steps: Optional[int] = None, warmup_rows: Optional[int] = None,
                          capacity: Optional[int] = None, log_every: int = 100,
                          use_graph: bool = True, stall_timeout_s: float = 60.0,
                          timeout_s: Optional[float] = None, ring_bytes: int = 256 << 20,
                          metrics_path: Optional[str] = None) -> Dict:
    """BASELINE config 2 topology: ONE learner process on the GPU (HBM replay, HIP learner) fed by
    ``n_actors`` CPU actor processes (the reference ``Actor`` with its env on the CPU) through the
    native transport -- shared-memory trajectory rings DMA'd into HBM (engine/ingest.py) and a
    shared-memory weight slot (parallel/weights.py ShmWeightsWriter) -- under the supervisor
    (dead / stalled actors are restarted as fresh processes)."""
    import uuid

    from .actor import actor_process
    from .engine.ingest import HBMIngestor
    from .engine.learner_engine import LearnerEngine
    from .engine.replay_hbm import HBMReplay
    from .parallel.dist import init_distributed
    from .parallel.weights import ShmWeightsWriter
    from .utils.metrics import MetricsLogger
    from .utils.supervisor import RoleSpec, Supervisor

    info = init_distributed()
    dev = info.device
    torch.manual_seed(cfg.seed)
    replay = HBMReplay(cfg, dev, capacity=capacity or cfg.replay.capacity, n_subrings=n_actors)
    eng = LearnerEngine(cfg, replay, dev)
    tag = f"{os.getpid()}_{uuid.uuid4().hex[:6]}"
    ring_names = [f"/r2d2_traj_{tag}_{i}" for i in range(n_actors)]
    ingest = HBMIngestor(replay, ring_names, ring_bytes=ring_bytes)
    wname = f"/r2d2_w_{tag}"
    weights = ShmWeightsWriter(wname, eng.layout.padded, dev)
    version = 0
    weights.publish(eng.master, eng.target, version)
    weights.poll(wait=True)
    roles = [RoleSpec(f"actor{i}", actor_process, (i, n_actors, None, "cpu"),
                      dict(cfg=cfg, shm_ring=ring_names[i], shm_weights=wname,
                           max_steps=actor_max_steps, seed=cfg.seed + 17 * i),
                      stall_timeout_s=stall_timeout_s) for i in range(n_actors)]
    sup = Supervisor(roles)
    mlog = MetricsLogger(metrics_path) if metrics_path else None
    warm = warmup_rows if warmup_rows is not None else min(cfg.learner.initial_exploration,
                                                           replay.capacity // 2)
    lc = cfg.learner
    out = {"steps": 0, "ingested_rows": 0, "records": 0}
    sup.start()
    t0 = time.perf_counter()
    t_ing = 0.0
    it = 0
    last_poll = 0.0
    captured = False
    t_train0 = None
    try:
        while it < steps:
            now = time.perf_counter()
            if timeout_s is not None and now - t0 > timeout_s:
                break
            if now - last_poll > 0.2:
                last_poll = now
                if not sup.poll():
                    break
            ta = time.perf_counter()
            got = ingest.poll()
            t_ing += time.perf_counter() - ta if got else 0.0
            if replay.total_written < warm or ingest.records == 0:
                if not got:
                    time.sleep(0.002)
                continue
            if not captured:
                if int(replay.n_valid.item()) < lc.batch_size:
                    time.sleep(0.002)
                    continue
                if use_graph and lc.use_graph:
                    eng.capture(warmup=1)
                captured = True
                t_train0 = time.perf_counter()
            eng.step()
            it += 1
            if it % lc.publish_interval == 0:
                version += 1
                weights.publish(eng.master, eng.target, version)
                eng.check_errors()
                ingest.check_errors()
            weights.poll()
            if it % log_every == 0 or it == steps:
                rec = dict(step=it, rows=ingest.rows, records=ingest.records,
                           learner_steps_per_s=it / (time.perf_counter() - t_train0), **eng.diagnostics())
                if mlog:
                    mlog.log("native_cpu", **rec)
                print("[native-cpu]", rec, flush=True)
        torch.cuda.synchronize(dev)
        eng.check_errors()
        ingest.check_errors()
    finally:
        sup.stop()
        ingest.close()
        weights.close()
    t_end = time.perf_counter()
    out.update(steps=it, ingested_rows=ingest.rows, records=ingest.records, ingest_bytes=ingest.bytes,
               wall_s=t_end - t0, ingest_host_s=t_ing,
               learner_steps_per_s=(it / (t_end - t_train0)) if t_train0 and it else 0.0,
               ingest_rows_per_s=ingest.rows / (t_end - t0), weights_version=version,
               # every ingested row is one CPU env step (the actors' aggregate env throughput)
               cpu_env_steps_per_s=ingest.rows / (t_end - t0),
               rejected_records=ingest.rejected, kernel_error_word=eng.error_word(),
               supervisor=sup.report, zero_copy=[b is not None for b in ingest.registered])
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
               stall_timeout_s: float = 0.0, learner_stall_timeout_s: float = 0.0) -> Dict:
    """Reference process topology under the supervisor.  Every role heartbeats (``beat``) and
    honours the fault hooks; a stalled learner (no beat for ``learner_stall_timeout_s``) stops the
    job, a dead / stalled actor is restarted as a fresh process."""
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
                      restartable=False, stall_timeout_s=learner_stall_timeout_s)]
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
