"""Batched GPU actor: device-side n-step returns, done flags, sequence starts, tree consistency;
native actor+learner loop; data-parallel engine consistency (2 ranks on one GPU over gloo)."""
import os
import socket

import numpy as np
import pytest
import torch

from pytorch_r2d2_amd.actor_batched import BatchedActor, PackedWeights, engine_weights
from pytorch_r2d2_amd.config import get_config
from pytorch_r2d2_amd.engine.layout import ParamLayout
from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
from pytorch_r2d2_amd.envs.synthetic import VecSyntheticAtari
from pytorch_r2d2_amd.models import QNet

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


class RecEnv(VecSyntheticAtari):
    """Records every step's rewards / dones into device logs (in place, so it also works when
    the actor replays its step as a HIP graph)."""

    def __init__(self, *a, max_steps=512, **k):
        super().__init__(*a, **k)
        self._r = torch.zeros(max_steps, self.E, device=self.device)
        self._d = torch.zeros(max_steps, self.E, dtype=torch.bool, device=self.device)
        self._i = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.steps = 0

    def step(self, actions):
        r, d, f = super().step(actions)
        self._r.index_copy_(0, self._i, r[None])
        self._d.index_copy_(0, self._i, d[None])
        self._i.add_(1)
        return r, d, f

    @property
    def log(self):
        n = int(self._i.item())
        return list(zip(self._r[:n].cpu().numpy(), self._d[:n].cpu().numpy()))


def _actor(E=8, cap_e=400, ep=37, graph=False, **over):
    kw = {"replay.burn_in": 4, "replay.learn": 6, "replay.overlap": 5, "replay.n_step": 3}
    kw.update(over)
    cfg = get_config("atari57", **kw)
    rp = HBMReplay(cfg, DEV, capacity=E * cap_e, n_subrings=E)
    torch.manual_seed(0)
    L = ParamLayout(cfg.model, cfg.env)
    w = PackedWeights(L, DEV)
    w.load(QNet("cpu", cfg.model, cfg.env).state_dict())
    env = RecEnv(E, DEV, seed=3, episode_len=ep, randomize_start=True)
    actor = BatchedActor(cfg, rp, env, w, w, seed=1)
    if graph:   # HIP-graph replay of the env step (the same checks must hold)
        assert actor.can_capture
        actor.capture(warmup=0)
    return cfg, rp, env, actor


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_actor_nstep_returns_dones_and_starts(graph):
    cfg, rp, env, actor = _actor(graph=graph)
    steps = 150
    actor.run(steps)
    torch.cuda.synchronize()
    n, g, T = cfg.replay.n_step, cfg.learner.gamma, cfg.replay.seq_len
    rew = np.stack([x[0] for x in env.log])      # (steps, E)
    dn = np.stack([x[1] for x in env.log])
    reward = rp.reward.cpu().numpy()
    done = rp.done.cpu().numpy()
    is_start = rp.is_start.cpu().numpy()
    E = env.E
    checked = 0
    for e in range(E):
        ep_first = 0
        ends = list(np.nonzero(dn[:, e])[0])
        for t in range(steps - n):
            # episode containing step t
            end = next((x for x in ends if x >= t), None)
            row = e * rp.cap_e + t
            if end is None:
                if t + n > steps - 1:
                    continue
                R = sum(g ** i * rew[t + i, e] for i in range(n))
                assert done[row] == 0
            else:
                m = min(n, end - t + 1)
                R = sum(g ** i * rew[t + i, e] for i in range(m))
                assert done[row] == (1 if end - t + 1 <= n else 0), (e, t, end)
            assert reward[row] == pytest.approx(R, rel=1e-5, abs=1e-5), (e, t)
            checked += 1
    assert checked > 500
    # every finished episode's return reached the (device) return ring
    rets = actor.finished_returns
    assert len(rets) == int(dn.sum()) > 0
    assert all(r == r and 0 <= r <= ep_len for r in rets for ep_len in [37])
    # starts: inside one episode, on the stride grid or the final start; window complete
    for e in range(E):
        ends = [-1] + list(np.nonzero(dn[:, e])[0])
        for s in np.nonzero(is_start[e * rp.cap_e:(e + 1) * rp.cap_e])[0]:
            ep0 = max(x for x in ends if x < s) + 1
            nxt = [x for x in ends if x >= s]
            assert (s - ep0) % cfg.replay.overlap == 0 or (nxt and s + T - 1 == nxt[0])
            if nxt:
                assert s + T - 1 <= nxt[0]
    # tree / counters consistent
    leaves = rp.tree[: rp.capacity]
    assert int(rp.n_valid.item()) == int(rp.is_start.sum().item()) > 0
    assert bool(((leaves > 0) == (rp.is_start > 0)).all())
    assert rp.total_priority() == pytest.approx(float(leaves.double().sum()), rel=1e-4)


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_actor_ring_wrap_invalidates_overwritten_sequences(graph):
    cfg, rp, env, actor = _actor(E=4, cap_e=60, ep=25, graph=graph)
    actor.run(200)   # > 3 passes over each sub-ring
    torch.cuda.synchronize()
    T, n = cfg.replay.seq_len, cfg.replay.n_step
    head = actor.head
    st = rp.is_start.cpu().numpy().reshape(4, rp.cap_e)
    for e in range(4):
        for s in np.nonzero(st[e])[0]:
            # a valid start's learning window never straddles the write head (new | old data)
            offs = (head - s) % rp.cap_e
            assert not (1 <= offs < T), (e, s, head)
    assert int(rp.n_valid.item()) == int(rp.is_start.sum().item())


def test_native_actor_learner_loop_runs():
    from pytorch_r2d2_amd.runner import run_native
    cfg = get_config("atari57", **{"learner.batch_size": 16, "replay.burn_in": 8, "replay.learn": 8,
                                   "replay.overlap": 8, "actor.envs_per_actor": 32,
                                   "env.episode_len": 60, "learner.initial_exploration": 3000})
    out = run_native(cfg, steps=30, log_every=10, capacity=32 * 300)
    assert len(out["losses"]) == 3 and all(np.isfinite(out["losses"]))
    assert out["env_steps"] > 3000


def test_native_loop_dmlab_rgb_runs():
    """DMLab-30 geometry (3x72x96 RGB) through actor + learner (library conv torso path)."""
    from pytorch_r2d2_amd.runner import run_native
    cfg = get_config("dmlab30", **{"learner.batch_size": 8, "replay.burn_in": 4, "replay.learn": 8,
                                   "replay.overlap": 6, "actor.envs_per_actor": 16,
                                   "env.episode_len": 40, "learner.initial_exploration": 800})
    out = run_native(cfg, steps=10, log_every=5, capacity=16 * 200)
    assert len(out["losses"]) == 2 and all(np.isfinite(out["losses"]))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, outdir, graph=False, same_data=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
    dist.init_process_group("gloo")
    cfg = get_config("atari57", **{"learner.batch_size": 8, "replay.burn_in": 4, "replay.learn": 4,
                                   "replay.overlap": 4, "learner.use_graph": False, "seed": 11})
    rp = HBMReplay(cfg, DEV, capacity=8 * 200, n_subrings=8)
    rp.fill_synthetic(episode_len=50, seed=0 if same_data else rank)   # different data per rank
    torch.manual_seed(5)
    eng = LearnerEngine(cfg, rp, DEV, rank=rank, world=world, process_group=dist.group.WORLD,
                        init_module=QNet("cpu", cfg.model, cfg.env))
    if same_data and rank == 0:
        # the same data on one rank (world 1, one graph / one eager sequence) for comparison
        rp1 = HBMReplay(cfg, DEV, capacity=8 * 200, n_subrings=8)
        rp1.fill_synthetic(episode_len=50, seed=0)
        torch.manual_seed(5)
        one = LearnerEngine(cfg, rp1, DEV, init_module=QNet("cpu", cfg.model, cfg.env))
        for _ in range(3):
            one.step_eager()
        torch.save({"master": one.master.cpu(), "loss": one.loss_value()},
                   os.path.join(outdir, "single.pt"))
    if graph:   # 4 graph segments with the bucket all-reduces issued between them
        eng.capture(warmup=1)
        steps = [eng.step] * 2
    else:
        steps = [eng.step_eager] * 3
    for fn in steps[:-1]:
        fn()
    torch.cuda.synchronize()
    root0, nv0 = float(rp.total_priority()), int(rp.n_valid.item())   # what the last step samples
    steps[-1]()
    torch.cuda.synchronize()
    torch.save({"master": eng.master.cpu(), "loss": eng.loss_value(), "probs": eng.probs.cpu(),
                "is_w": eng.is_w.cpu(), "dp_params": eng.dp_params.cpu(), "dp_recv": eng.dp_recv.cpu(),
                "root": root0, "n_valid": nv0,
                "beta": float(cfg.replay.beta), "dp_global": eng.dp_global},
               os.path.join(outdir, f"dp{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_dp_engine_ranks_stay_identical(tmp_path, graph):
    import torch.multiprocessing as tmp
    tmp.spawn(_dp_worker, args=(2, _free_port(), str(tmp_path), graph), nprocs=2, join=True)
    a = torch.load(tmp_path / "dp0.pt", weights_only=True)
    b = torch.load(tmp_path / "dp1.pt", weights_only=True)
    assert torch.equal(a["master"], b["master"])       # synchronous DP: identical replicas
    assert a["loss"] != b["loss"]                       # ...trained on different local batches


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_dp_engine_on_identical_shards_matches_single_rank(tmp_path, graph):
    """Two ranks on identical replay shards = one rank: the DP step order (core bucket beside the
    conv backward, priority refresh + tree repair beside the torso bucket, then update + step
    counter) must reproduce the single-rank trajectory, sampling included."""
    import torch.multiprocessing as tmp
    tmp.spawn(_dp_worker, args=(2, _free_port(), str(tmp_path), graph, True), nprocs=2, join=True)
    a = torch.load(tmp_path / "dp0.pt", weights_only=True)
    one = torch.load(tmp_path / "single.pt", weights_only=True)
    torch.testing.assert_close(a["master"], one["master"], rtol=0, atol=1e-6)
    assert abs(a["loss"] - one["loss"]) <= 1e-5 * max(1.0, abs(one["loss"]))


def test_native_loop_learns_synthetic_cue_task():
    """End to end: batched GPU actor + HIP learner (both as HIP graphs) learn the synthetic cue
    task (reward 1 when the action matches the bright column band).  A random policy returns
    episode_len / n_actions; after 1500 learner steps the greedy-ish policy must be far above."""
    from pytorch_r2d2_amd.runner import run_native
    ep = 64
    cfg = get_config("atari57", **{
        "learner.batch_size": 32, "replay.burn_in": 8, "replay.learn": 16, "replay.overlap": 8,
        "replay.n_step": 3, "actor.envs_per_actor": 64, "env.episode_len": ep,
        "learner.initial_exploration": 4000, "learner.lr": 2.5e-4, "learner.optimizer": "adam",
        "learner.target_update_interval": 200, "learner.gamma": 0.9})
    out = run_native(cfg, steps=1500, log_every=500, capacity=64 * 1000)
    rets = np.asarray(out["returns"])
    random_return = ep / cfg.model.n_actions
    assert len(rets) > 500
    assert rets[-200:].mean() > 3 * random_return, (rets[:200].mean(), rets[-200:].mean())


def _memory_task(ablation: str, steps: int, extra=()):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    from learn_check import make_cfg, memoryless_ceiling, parse
    from pytorch_r2d2_amd.runner import run_native
    args = parse(["--memory", "--ablation", ablation, "--steps", str(steps), *extra])
    cfg = make_cfg(args, "fp32")
    out = run_native(cfg, steps=steps, log_every=steps, capacity=args.envs * 1000)
    rets = np.asarray(out["returns"])
    return rets, memoryless_ceiling(args.episode_len, args.switch, cfg.model.n_actions)


def test_recurrent_learner_solves_memory_task():
    """The cue is drawn only on the first frame after each target switch (env.cue_only_first,
    switch 8), so a memoryless policy returns at most (1/8 + 7/8 * 1/6) * 64 = 17.3 per episode.
    The fp32 learner (stored state + burn-in + BPTT over 16 learned steps, the atari57 engine
    path) must carry the target in its LSTM state: >= 2x that ceiling
    (profiles/r03_learn_memory_task.txt: 60.4 = 3.5x after 8000 steps)."""
    rets, ceil = _memory_task("none", 4000)
    assert len(rets) > 1000
    assert rets[-300:].mean() >= 2.0 * ceil, (rets[:300].mean(), rets[-300:].mean(), ceil)


def test_stored_state_beats_zero_state_on_long_memory():
    """What stored recurrent state + burn-in buy (/root/reference/learner.py:71-79,
    replay_memory.py:238-241): the cue is shown once per 64-step target phase, the training
    window is 4 burn-in + 8 learned steps, so a learner that starts every sequence from a zero
    state (no burn-in, 12 learned steps) never sees the cue in most windows and cannot learn to
    hold it for 63 steps; the full learner starts from the actors' stored states.  Full must beat
    zero-state by >= 1.3x (profiles/r04_learn_stored_state.txt: 115.6 vs 64.5 after 8000 steps)."""
    extra = ("--switch", "64", "--episode-len", "128", "--burn-in", "4", "--learn", "8")
    full, ceil = _memory_task("none", 6000, extra)
    zero, _ = _memory_task("zero_state", 6000, extra)
    assert len(full) > 1000 and len(zero) > 1000
    f, z = full[-300:].mean(), zero[-300:].mean()
    assert f >= 1.3 * z and f >= 2.0 * ceil, (f, z, ceil)


def test_memoryless_ablation_stays_at_ceiling():
    """Ablation of the same task: LSTM state reset before every actor step, learner sequences
    of one step from a zero state -- no memory anywhere, so the return stays near the ceiling."""
    rets, ceil = _memory_task("memoryless", 4000)
    assert len(rets) > 1000
    assert rets[-300:].mean() <= 1.15 * ceil, (rets[-300:].mean(), ceil)


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_dp_engine_global_sampling_weights(tmp_path, graph):
    """Different shards per rank: the TD kernel's IS weights are the two-level global ones
    (parallel/sharded_replay.py) computed from the all-gathered shard stats."""
    from pytorch_r2d2_amd.parallel.sharded_replay import dp_is_weights, global_is_params
    import torch.multiprocessing as tmp
    tmp.spawn(_dp_worker, args=(2, _free_port(), str(tmp_path), graph), nprocs=2, join=True)
    r = [torch.load(os.path.join(tmp_path, f"dp{k}.pt"), weights_only=True) for k in range(2)]
    assert r[0]["dp_global"] and r[1]["dp_global"]
    stats = r[0]["dp_recv"].view(2, 3)
    torch.testing.assert_close(stats, r[1]["dp_recv"].view(2, 3))
    for k in range(2):
        assert abs(float(stats[k, 0]) - r[k]["root"]) <= 1e-5 * r[k]["root"]
        assert int(stats[k, 1]) == r[k]["n_valid"]
        assert float(stats[k, 2]) == float(r[k]["probs"].min())
        params = global_is_params(stats, k, r[k]["beta"])
        torch.testing.assert_close(r[k]["dp_params"], params, rtol=1e-6, atol=0)
        torch.testing.assert_close(r[k]["is_w"], dp_is_weights(r[k]["probs"], params, r[k]["beta"]),
                                   rtol=2e-6, atol=1e-7)
    assert max(float(r[k]["is_w"].max()) for k in range(2)) == pytest.approx(1.0, rel=1e-6)


@pytest.mark.parametrize("cue_only_first", [False, True])
def test_fused_synthetic_env_step_dynamics(cue_only_first):
    """csrc/kernels/env.hip (one launch per step of all E envs) against the env's rules: reward =
    (action == target before the step), episode counter / auto-reset / finished returns, targets
    redrawn only on switch steps, and the rendered observation: the target's column band at 220
    exactly when the cue is shown, noise in 0..47 everywhere else."""
    E, A, ep, sw = 32, 6, 19, 4
    env = VecSyntheticAtari(E, DEV, seed=5, episode_len=ep, n_actions=A, switch=sw,
                            cue_only_first=cue_only_first)
    assert env.fused
    env.reset_all()
    g = torch.Generator(device=DEV).manual_seed(1)
    ret = torch.zeros(E, device=DEV)
    band = 84 // A
    cols = torch.arange(84, device=DEV)
    for _ in range(3 * ep):
        t0, tgt0 = env.t.clone(), env.target.clone()
        act = torch.randint(0, A, (E,), device=DEV, generator=g)
        r, d, f = env.step(act)
        exp_r = (act == tgt0).float()
        assert torch.equal(r, exp_r)
        t1 = t0 + 1
        assert torch.equal(d, t1 >= ep)
        ret += exp_r
        fin = torch.where(d, ret, torch.full_like(ret, float("nan")))
        assert torch.equal(torch.isnan(f), torch.isnan(fin)) and torch.equal(f[d], fin[d])
        ret[d] = 0
        assert torch.equal(env.t, torch.where(d, torch.zeros_like(t1), t1))
        keep = (t1 % sw) != 0
        assert torch.equal(env.target[keep], tgt0[keep])
        assert int(env.target.min()) >= 0 and int(env.target.max()) < A
        fr = env.frames.view(E, 4, 84, 84)
        in_band = (cols[None, :] // band == env.target[:, None]) & (cols[None, :] < band * A)   # (E, W)
        show = torch.ones(E, dtype=torch.bool, device=DEV) if not cue_only_first else (env.t % sw) == 0
        m = (in_band & show[:, None])[:, None, None, :].expand_as(fr)
        assert bool((fr[m] == 220).all())
        assert int(fr[~m].max()) <= 47
    noise = env.frames.view(E, 4, 84, 84).float()
    assert 20.0 < float(noise[noise <= 47].mean()) < 27.0


def _force_dp_worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    import torch.distributed as dist
    from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    out = {}
    for force, one in ((True, False), (True, True), (False, False)):
        cfg = get_config("atari57", **{"learner.batch_size": 8, "replay.burn_in": 4,
                                       "replay.learn": 4, "replay.overlap": 4, "seed": 11,
                                       "learner.use_graph": False, "dist.force_dp": force,
                                       "dist.graph_collectives": one})
        rp = HBMReplay(cfg, DEV, capacity=8 * 200, n_subrings=8)
        rp.fill_synthetic(episode_len=50, seed=0)
        torch.manual_seed(5)
        eng = LearnerEngine(cfg, rp, DEV, process_group=dist.group.WORLD if force else None,
                            init_module=QNet("cpu", cfg.model, cfg.env))
        assert eng.dp == force and eng.dp_global == force
        eng.capture(warmup=1)
        if force:       # the segment graphs; the one graph after dist.one_graph_warm steps
            assert len(eng.graphs) == 6
        for _ in range(5):
            eng.step()
        torch.cuda.synchronize()
        assert eng.error_word() == 0
        if force:
            assert eng._rollout.mode == ("one" if one else "segments"), eng.dp_graph_label()
        out[(force, one)] = {"master": eng.master.cpu(), "loss": eng.loss_value()}
    torch.save(out, os.path.join(outdir, "force_dp.pt"))
    dist.destroy_process_group()


def test_forced_dp_step_over_rccl_matches_plain_step(tmp_path):
    """The N-GPU step machinery at ONE rank over RCCL (dist.force_dp): six graph segments, the
    bucketed all-reduces on the comm stream and the shard-stats all-gather as one-rank
    collectives, then (dist.graph_collectives) the one captured graph after the warm-up steps --
    the same trajectory as the plain single-rank step (what the 8-GPU run uses, exercised on the
    real backend instead of gloo)."""
    import torch.multiprocessing as tmp
    tmp.spawn(_force_dp_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    r = torch.load(tmp_path / "force_dp.pt", weights_only=True)
    plain = r[(False, False)]
    for key in ((True, False), (True, True)):     # segmented graphs; one graph, RCCL captured
        torch.testing.assert_close(r[key]["master"], plain["master"], rtol=0, atol=1e-6)
        assert abs(r[key]["loss"] - plain["loss"]) <= 1e-5 * max(1.0, abs(plain["loss"]))
