"""Typed configuration for the MI355X-native R2D2 engine.

The reference hard-codes every hyper-parameter as a literal inside class constructors
(``/root/reference/actor.py:21-51``, ``learner.py:20-51``, ``replay_memory.py:59-74``) and
exposes a single CLI flag (``main.py:14``).  Here every knob lives in one dataclass tree with
named presets:

* ``reference``   -- the exact values of the reference: B=8, burn-in 10 + learn 10,
                     n=3, gamma=0.99, centered RMSprop, Pong network.
* ``cartpole``    -- CartPole-v1 plumbing config (seq 80 / burn-in 40) on CPU (BASELINE config 1).
* ``pong``        -- Pong, 1 MI355X learner + 64 actor envs, replay resident in HBM (config 2).
* ``atari57``     -- the R2D2 paper shapes: B=64, burn-in 40 + learn 40, n=5, gamma=0.997,
                     value rescaling, IS weights (config 3).  This is the ``bench.py`` headline.
* ``seaquest8``   -- 8-GPU data-parallel learner + 512 actor envs (config 4).
* ``dmlab30``     -- 96x72 RGB synthetic frames, bf16 LSTM, sharded replay (config 5).
"""
from __future__ import annotations

import copy
import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class EnvConfig:
    name: str = "synthetic"          # synthetic | cartpole | pong | dmlab_synth
    action_repeat: int = 4            # env.py:15
    n_stacks: int = 4                 # env.py:15
    frame_h: int = 84
    frame_w: int = 84
    channels_per_frame: int = 1       # 1 = gray (Atari), 3 = RGB (DMLab)
    n_actions: int = 6                # model.py:35 (Pong)
    episode_len: int = 400            # synthetic env only
    # synthetic cue task: the rewarded action changes every ``switch`` agent steps; with
    # ``cue_only_first`` its cue is drawn only on the first frame after a change, so acting well
    # needs memory (a memoryless policy scores (1/switch + (1 - 1/switch)/A) per step)
    switch: int = 8
    cue_only_first: bool = False
    obs_dim: int = 4                  # vector envs (CartPole)


@dataclass
class ModelConfig:
    torso: str = "atari"              # atari | mlp
    conv_channels: tuple = (32, 32, 32)   # model.py:14-20 (comments say 16/32/64; code is 32/32/32)
    hidden: int = 256                 # model.py:24
    head_hidden: int = 256            # model.py:27,33
    mlp_hidden: int = 64              # mlp torso width (CartPole)
    n_actions: int = 6


@dataclass
class ReplayConfig:
    capacity: int = 500_000           # learner.py:38
    burn_in: int = 10                 # learner.py:35
    learn: int = 10                   # learner.py:36
    overlap: int = 10                 # actor.py:40 (stride between sequence starts)
    n_step: int = 3                   # learner.py:23
    eta: float = 0.9                  # replay_memory.py:71
    alpha: float = 0.6                # actor.py:24 / learner.py:22
    priority_eps: float = 1e-6        # learner.py:25
    beta: float = 0.0                 # IS exponent; 0 == reference (no IS weights, Q10)
    stored_state: str = "post"        # post == reference (Q6); pre == paper
    n_subrings: int = 1               # one contiguous sub-ring per actor env (HBM replay)
    # learner tail: sum-tree levels >= 2 and the step counter folded into the level-1 repair
    # launch (last-arriving workgroup), 2 launches instead of levels - 1 + 1
    fused_tree_tail: bool = True
    # ... and the sequence-priority refresh + level-0 repair in the same launch (grid barriers
    # between the levels, replay.hip prio_tail_kernel): the whole priority tail is one launch
    fused_prio_tail: bool = True

    @property
    def seq_len(self) -> int:
        return self.burn_in + self.learn


@dataclass
class LearnerConfig:
    batch_size: int = 8               # learner.py:39
    gamma: float = 0.99               # learner.py:21
    optimizer: str = "rmsprop_centered"   # learner.py:51 ; or "adam" (paper)
    lr: float = 0.00025 / 4.0
    rms_alpha: float = 0.95
    eps: float = 1.5e-7
    adam_betas: tuple = (0.9, 0.999)
    grad_clip: float = 0.0            # 0 == off (reference)
    value_rescale: bool = False       # h(x) = sign(x)(sqrt(|x|+1)-1)+eps*x  (paper)
    value_rescale_eps: float = 1e-3
    target_update_interval: int = 1000    # learner.py:46
    publish_interval: int = 100       # learner.py:45
    ingest_interval: int = 20         # learner.py:40
    checkpoint_interval: int = 10_000     # learner.py:117
    initial_exploration: int = 50_000     # learner.py:24
    # "reference": 3 recurrent chains exactly like learner.py:75-93 (online on state, target on
    # next_state, online on next_state continuing the learning chain's state -- Q7 reproduced).
    # "fixed": Q7 fixed -- online-on-next gets its own stored state + burn-in.
    # "shifted": R2D2 paper form -- one online and one target chain over T+n frames;
    #            Q(s_{t+n}) is read at offset +n of the same chain.
    target_mode: str = "shifted"
    # "fp32": the reference's precision (fp32 weights/activations/state; MFMA products as three
    # bf16 passes over hi/lo splits, csrc/split.h) | "bf16": bf16 operands, fp32 accumulate
    compute_dtype: str = "bf16"
    lstm_impl: str = "persistent"     # persistent (one launch per sequence) | step (launch per t)
    # persistent forward hand-off: "tagged" (8-byte {h pair, tag} granules polled directly, 16-row
    # batch tiles; falls back when the grid does not fit) | "counter" (payload + arrival counter)
    lstm_handoff: str = "tagged"
    # post-BPTT GEMMs: "group" = weight gradients + dX in one grid (58 us vs 85 separate),
    # "group:a,b,c,d" = with K splits, "separate"
    bwd_gemm: str = "group"
    # rmsprop writes the LSTM / head row packs itself (optim.hip rmsprop_pack_kernel) instead of
    # a gather over the updated master in the pack launch
    fuse_opt_pack: bool = True
    # world 1: the torso backward's slab reduction folded into that optimizer launch (its first
    # workgroups; optim.hip r2_rmsprop_pack_slab) instead of its own torso_grad_reduce launch
    fold_torso_reduce: bool = True
    td_fuse_head_bwd: bool = True     # dueling-head backward inside the TD launch (td_duel_kernel)
    # ... and the heads' dueling FORWARD too (fixed / reference target modes: the TD launch forms
    # relu(z + b1) and the Q rows of all three heads itself; no separate dueling_fwd launch)
    td_fuse_head_fwd: bool = True
    # ... and the head's input gradient dh = dz @ W1 on that launch's MFMAs (hidden 256): no
    # separate dh GEMM (hipBLASLt 7-10 us in bf16, 22 us split-precision)
    td_fuse_dh: bool = True
    # tagged LSTM forward with 9..16 groups (fixed target: 3 chains x 4 batch tiles) placed two
    # groups per XCD, so every group's h hand-off stays in one XCD's L2 (else spread over all XCDs:
    # write-through stores, fabric-latency polls)
    lstm_xcd_pairs: bool = True
    # split precision (compute_dtype fp32) GEMMs: "fused" = gemm_sp.hip (hi / lo planes staged
    # once, 3 MFMAs per fragment pair: x-projection 164 -> 125 us, post-BPTT group 142 -> 106 us
    # at K splits 4,4,4,1, dh 26 -> 18 us; profiles/archive/r02_gemm_sp_micro_v1.txt) | "multipass"
    sp_gemm: str = "fused"
    # K splits of the fused post-BPTT group (dW_ih, dW_hh, dW_head1, dX), or "auto"
    # (learner_engine._auto_group_splits: paper config 4,4,4,1, reference config 1,1,1,4)
    sp_group_splits: str = "auto"
    # tile config of that group: ops/gemm.py G5_CFGS index, -1 = the launcher's CU model, -2 =
    # learner_engine._auto_group_splits' choice (paper shape: 128x128, 4-deep 32-K ring)
    sp_group_cfg: int = -2
    # split precision: the dueling head's gradient reduction on the BPTT launch's idle workgroups
    # (r2_lstm_bwd_tag_sp_hg) instead of its own 28 us launch
    sp_head_grads_in_bptt: bool = True
    torso_bwd: str = "fused"         # fused (HIP kernel) | library (MIOpen convolution_backward)
    # library conv path (frame geometries without the fused HIP torso, e.g. DMLab): MIOpen find
    # mode (torch.backends.cudnn.benchmark) instead of its immediate-mode heuristics
    conv_autotune: bool = True
    use_graph: bool = True            # capture the whole step in a HIP graph
    # split precision: the BPTT computes its input gradient dh = dz . W1 itself, inside its
    # hand-off waits (lstm_persist.hip PTBArgs::dz), instead of the TD launch (td_fuse_dh)
    bptt_dh: bool = True
    # (round 5's post-BPTT GEMMs on the BPTT launch's idle workgroups -- learner.bptt_gemms --
    # slowed the recurrence in every arm and were removed: profiles/r05_bptt_helpers_roles.txt)
    # Single-rank split-precision step, software-pipelined over two steps (learner_engine.py
    # "hoisted step"): right after step k's TD launch a side stream runs step k's priority tail,
    # step k+1's sample and step k+1's target-network torso frames on the CUs the BPTT leaves
    # free (a frame queue the next step's torso launch finishes); bit-identical to the plain step
    hoist: bool = True
    # the BPTT raises the side torso's stop word this many iterations before its last one (the
    # side workgroups finish the frame in hand and the one already taken: ~1.5 frames)
    hoist_stop_lead: int = 5
    # hoisted step, graph mode: LearnerEngine.run_steps(n) replays runs of this many consecutive
    # steps (no target sync inside, the previous step sampled) as ONE captured graph, so the
    # ~5 us boundary between two graph replays is paid once per chunk; 1 = a graph per step
    graph_chunk: int = 8
    # hoisted step: fork the side branch before the TD launch instead of after it; the priority
    # tail, launched beside TD, waits for TD's done flag on the device (td.hip TdDuelArgs::done)
    hoist_early_fork: bool = True
    # (removed A/B knobs whose alternative lost, record in profiles/: lstm_tag_words = False, the
    # 8-byte hand-off granules (archive/bench_r02_tag_words_ab.log); sp_gemm6 = False, gemm5
    # (r03_gemm6_ab.txt); sp_gemm_order = 0 (r05_gemm_item_order.txt); sp_heads_cfg
    # (r03_heads_cfg_ab.txt); torso_save_weight 1.15 / 1.3, hoist_full_repack, hoist_join "end",
    # hoist_avoid_xcds, bptt_hg_wgs 64, bptt_xcd_pairs off (r06_tree_ab_knobs.txt,
    # r06_hoist_knobs_rejected.txt))
    # single-rank step: the weight repack after the optimizer (pack_step) runs on extra
    # workgroups of the priority tail's launch (replay.hip r2_prio_tail_pack): one launch fewer
    fuse_pack_tail: bool = True
    save_dir: str = "save"
    # ablation (tools/learn_check.py): ignore the stored recurrent state of every sampled
    # sequence (zeros instead of the actor's (h, c)); with burn_in = 0 the learner has no context
    # from before the sequence start
    zero_stored_state: bool = False


@dataclass
class ActorConfig:
    n_actors: int = 1                 # main.py:14
    envs_per_actor: int = 1
    eps_base: float = 0.4             # actor.py:22
    eps_alpha: float = 7.0
    net_load_interval: int = 5        # actor.py:51 (episodes)
    memory_save_interval: int = 5     # actor.py:44 (episodes)
    local_capacity: int = 50_000      # actor.py:34
    # batched GPU actor: replay each env step as a HIP graph (two variants: plain / sub-ring
    # wrap); needs a device env whose step() is capture-safe (VecSyntheticAtari)
    use_graph: bool = True
    return_ring: int = 4096           # device ring of finished-episode returns (drained lazily)
    # ablation (tools/learn_check.py): reset both nets' LSTM state before every env step -- a
    # memoryless acting policy (with seq_len 1 and zeroed stored state, a memoryless learner)
    reset_state_every_step: bool = False


@dataclass
class DistConfig:
    backend: str = "auto"             # nccl (RCCL) on GPU, gloo on CPU
    grad_bucket_mb: float = 8.0
    grad_dtype: str = "fp32"          # fp32 | bf16 (compressed all-reduce)
    overlap_allreduce: bool = True
    # CUs the fused conv backward leaves free while the core gradient bucket is being all-reduced
    # (world > 1): torso_bwd_kernel fills every VGPR of each CU it runs on (248 VGPRs x 8 waves),
    # so without a reservation the RCCL kernel cannot start until the conv backward has finished
    # (no overlap at all).  0 = whole chip (the world == 1 layout).
    comm_reserve_cus: int = 32
    # globally proportional prioritized sampling over the ranks' replay shards
    # (parallel/sharded_replay.py: one 12-byte all-gather per step, shard-ratio loss weights)
    global_sampling: bool = True
    # split topology (parallel/actor_ranks.py, runner.run_split): the last ``actor_ranks`` ranks
    # run actor groups only and feed the learner ranks over asynchronous RCCL links; every
    # ``push_rows`` env steps an actor rank ships one record of its newest final rows (each row
    # once), blocking only when ``push_slots`` records are untaken; learner rank 0 sends weights
    # every ``publish_steps`` learner steps to the actor ranks that took the previous snapshot
    actor_ranks: int = 0
    push_rows: int = 32
    push_slots: int = 4
    publish_steps: int = 100
    # the learner reads its links' ``sent`` counters (one c10d store round trip per feeding actor
    # rank, served by rank 0) at most every ``poll_steps`` learner steps once it is training; an
    # actor rank ships a record every push_rows env steps, so polling every step only adds host
    # latency to the step loop (before training starts every iteration polls)
    poll_steps: int = 8
    # rehearsal: run the data-parallel step machinery (segmented graphs, bucketed RCCL
    # all-reduces on the comm stream, CU reservation, the shard-stats all-gather) at world 1
    # (bench.py --force-dp under torchrun): the collectives are one-rank no-ops, the code path is
    # the N-GPU one
    force_dp: bool = False
    # capture the DP step as ONE graph, the RCCL collectives included (side-stream fork / join
    # edges), instead of 4-6 segment graphs with the collectives issued between them: the DP
    # machinery's overhead at one forced rank 1.180 -> 1.122 ms against 1.102 for the plain step
    # (tools/dp_overhead_ab.sh, profiles/r03_force_dp_ab.txt)
    graph_collectives: bool = True
    # ... also at world > 1, rolled out per run (parallel/graph_rollout.py): the first
    # one_graph_warm steps replay the segment graphs, then the one graph with a one_graph_validate
    # step window in which every rank records a weight checksum + its error word on the device,
    # checked by ONE all-reduce at the window's end; any mismatch sends every rank back to the
    # segment graphs (rank 0's state re-broadcast) and bench.py labels the run
    graph_collectives_multi: bool = True
    one_graph_warm: int = 3
    one_graph_validate: int = 50
    learner_steps_per_round: int = 1    # run_split default run length: rounds x this


@dataclass
class R2D2Config:
    name: str = "reference"
    env: EnvConfig = field(default_factory=EnvConfig)
    model: ModelConfig = field(default_factory=ModelConfig)
    replay: ReplayConfig = field(default_factory=ReplayConfig)
    learner: LearnerConfig = field(default_factory=LearnerConfig)
    actor: ActorConfig = field(default_factory=ActorConfig)
    dist: DistConfig = field(default_factory=DistConfig)
    seed: int = 0

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def replace(self, **overrides) -> "R2D2Config":
        """Return a copy with dotted overrides, e.g. ``replace(**{"learner.batch_size": 64})``."""
        cfg = copy.deepcopy(self)
        for key, val in overrides.items():
            apply_override(cfg, key, val)
        return cfg


def apply_override(cfg: R2D2Config, dotted: str, value: Any) -> None:
    parts = dotted.split(".")
    obj = cfg
    for p in parts[:-1]:
        obj = getattr(obj, p)
    cur = getattr(obj, parts[-1])
    if isinstance(value, str) and not isinstance(cur, str):
        if isinstance(cur, bool):
            value = value.lower() in ("1", "true", "yes", "on")
        elif isinstance(cur, int):
            value = int(value)
        elif isinstance(cur, float):
            value = float(value)
        elif isinstance(cur, tuple):
            value = tuple(type(cur[0])(v) for v in value.split(","))
    setattr(obj, parts[-1], value)


def _reference() -> R2D2Config:
    c = R2D2Config(name="reference")
    # the reference's 3-chain target structure (learner.py:71-93) with Q7 fixed, at the
    # reference's precision (fp32 end to end: model.py / learner.py use no reduced precision)
    c.learner.target_mode = "fixed"
    c.learner.compute_dtype = "fp32"
    return c


def _cartpole() -> R2D2Config:
    c = R2D2Config(name="cartpole")
    c.env = EnvConfig(name="cartpole", action_repeat=1, n_stacks=1, n_actions=2, obs_dim=4,
                      episode_len=500)
    c.model = ModelConfig(torso="mlp", hidden=64, head_hidden=64, mlp_hidden=64, n_actions=2)
    c.replay = ReplayConfig(capacity=100_000, burn_in=40, learn=40, overlap=40, n_step=5,
                            beta=0.6, stored_state="pre")
    c.learner = LearnerConfig(batch_size=16, gamma=0.997, optimizer="adam", lr=1e-3, eps=1e-3,
                              value_rescale=True, target_update_interval=100,
                              initial_exploration=2_000, compute_dtype="fp32", use_graph=False)
    c.actor = ActorConfig(n_actors=1, envs_per_actor=16)
    return c


def _pong() -> R2D2Config:
    c = R2D2Config(name="pong")
    c.env = EnvConfig(name="synthetic", n_actions=6)
    c.replay = ReplayConfig(capacity=2_000_000, n_subrings=64)
    # the reference's own game: its precision (fp32) and its 3-chain target structure with Q7
    # fixed (learner.py:71-93), like the ``reference`` preset
    c.learner = LearnerConfig(batch_size=8, target_mode="fixed", compute_dtype="fp32")
    c.actor = ActorConfig(n_actors=1, envs_per_actor=64)
    return c


def _atari57() -> R2D2Config:
    c = R2D2Config(name="atari57")
    c.env = EnvConfig(name="synthetic", n_actions=6)
    c.model = ModelConfig(n_actions=6)
    c.replay = ReplayConfig(capacity=1_000_000, burn_in=40, learn=40, overlap=40, n_step=5,
                            eta=0.9, alpha=0.9, beta=0.6, stored_state="pre", n_subrings=256)
    c.learner = LearnerConfig(batch_size=64, gamma=0.997, optimizer="rmsprop_centered",
                              value_rescale=True, target_update_interval=2500,
                              target_mode="fixed", compute_dtype="fp32")
    c.actor = ActorConfig(n_actors=1, envs_per_actor=256)
    return c


def _seaquest8() -> R2D2Config:
    c = _atari57()
    c.name = "seaquest8"
    c.env.n_actions = 18
    c.model.n_actions = 18
    c.actor = ActorConfig(n_actors=8, envs_per_actor=64)
    c.replay.n_subrings = 64
    return c


def _dmlab30() -> R2D2Config:
    c = _atari57()
    c.name = "dmlab30"
    c.env = EnvConfig(name="dmlab_synth", action_repeat=4, n_stacks=1, frame_h=72, frame_w=96,
                      channels_per_frame=3, n_actions=15)
    c.model.n_actions = 15
    c.actor = ActorConfig(n_actors=8, envs_per_actor=64)
    # BASELINE config 5 names a bf16 LSTM for DMLab; the split-precision mode needs the fused
    # Atari torso
    c.learner.compute_dtype = "bf16"
    return c


PRESETS = {
    "reference": _reference,
    "cartpole": _cartpole,
    "pong": _pong,
    "atari57": _atari57,
    "seaquest8": _seaquest8,
    "dmlab30": _dmlab30,
}


def get_config(name: str = "reference", **overrides) -> R2D2Config:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name!r}; choose from {sorted(PRESETS)}")
    cfg = PRESETS[name]()
    return cfg.replace(**overrides) if overrides else cfg


def epsilon_ladder(actor_id: int, n_actors: int, base: float = 0.4, alpha: float = 7.0) -> float:
    """Ape-X per-actor epsilon ``base ** (1 + alpha * i / (N - 1))`` (``actor.py:22``).

    Fix for Q1: the reference divides by zero when ``N == 1``; a single actor gets ``base``.
    """
    if n_actors <= 1:
        return base
    return base ** (1.0 + alpha * actor_id / (n_actors - 1))
