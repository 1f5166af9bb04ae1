"""The hoisted learner step (learner.hoist, engine/learner_engine.py "hoisted step"): step k's
priority tail, step k+1's sample and part of step k+1's target-network torso run on a side stream
beside step k's BPTT.  It must be bit-identical to the plain serial step (the reference's train
order, /root/reference/learner.py:68-110), target syncs included."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _engine(hoist, B=64, interval=3, graph=True, **kw):
    from pytorch_r2d2_amd.config import get_config
    from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    over = {"seed": 1234, "learner.batch_size": B, "learner.hoist": hoist,
            "learner.target_update_interval": interval, "learner.use_graph": graph}
    over.update(kw)
    cfg = get_config("atari57", **over)
    rp = HBMReplay(cfg, DEV, capacity=64000)
    rp.fill_synthetic(episode_len=200, seed=3)
    eng = LearnerEngine(cfg, rp, DEV)
    return rp, eng


def _state(rp, eng):
    # the packed layouts by name (their alignment padding is never read and not compared)
    out = {"master": eng.master, "target": eng.target, "opt_a": eng.opt_a, "opt_b": eng.opt_b,
           "lstm_b": eng.lstm_b, "lstm_b_t": eng.lstm_b_t, "priority": rp.priority,
           "tree": rp.tree, "step": rp.step, "loss": eng.loss}
    for tag, (bf, f32) in {"": (eng.bf, eng.f32), "_t": (eng.bf_t, eng.f32_t)}.items():
        for plane in range(bf.shape[0]):
            for k, v in eng.layout.packed_views(bf[plane], f32).items():
                out["%s%s.%d" % (k, tag, plane)] = v
    return out


@pytest.mark.parametrize("graph,B,early", [(True, 64, False), (False, 64, False), (True, 16, False),
                                           (False, 8, False), (True, 64, True), (False, 16, True)])
def test_hoisted_step_is_bitwise_the_plain_step(graph, B, early):
    """Bench shape (B=64, 40 + 40, n=5, fixed target), target sync every 3 steps (steps 2, 5, 8
    sync: the step after each runs the full target torso), one invalidation in the middle (the
    next step samples at its start): weights, optimizer moments, every packed layout, priorities,
    sum tree and step counter equal the plain engine's after every step; error word 0.  B 8 / 16:
    one batch tile, an odd count of recurrence groups packed in XCD pairs (the head-gradient
    helpers' ordinals, lstm_persist.hip xcd_map 3).  ``early``: the side branch forks before the
    TD launch and its priority tail waits for TD's done flag on the device."""
    rp0, plain = _engine(False, B=B, graph=graph)
    rp1, hoist = _engine(True, B=B, graph=graph, **{"learner.hoist_early_fork": early})
    assert hoist.hoist and not plain.hoist
    if graph:
        plain.capture(warmup=0)
        hoist.capture(warmup=0)
    for i in range(10):
        if i == 6:
            hoist.invalidate_hoist()
        plain.step()
        hoist.step()
        torch.cuda.synchronize()
        a, b = _state(rp0, plain), _state(rp1, hoist)
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        assert not bad, (i, bad)
    assert plain.error_word() == 0 and hoist.error_word() == 0
    assert torch.equal(plain.starts, hoist.starts)


def test_hoisted_side_torso_takes_frames():
    """In steady state the side stream's torso launch really computes target frames (queue word 0
    > 0 after a non-sync step) and the next torso launch takes the rest (word 1)."""
    rp, eng = _engine(True, interval=1000)
    eng.capture(warmup=1)
    for _ in range(4):
        eng.step()
    torch.cuda.synchronize()
    q = eng.tq.cpu().tolist()
    n = (eng.Tn - eng.t_lo_tg) * eng.B
    assert 0 < min(q[0], n) < n, q      # side frames; the rest left to the next launch
    assert q[2] == 1                    # the BPTT raised its stop word
    assert eng.error_word() == 0


def test_torso_queue_jobs_match_static_job():
    """torso_sp.hip queue jobs: a qmode-1 launch stopped part-way, then a qmode-2 launch beside
    static jobs (device-side deal), produce the same features bitwise as one static launch."""
    from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle
    rp, eng = _engine(True, B=16, graph=False)
    eng._sample()
    torch.cuda.synchronize()
    k = kernels()
    pt, ptl = eng.pk_t, eng.pk_t_lo
    rows = eng.rows[eng.t_lo_tg * eng.B:]
    n = rows.numel()
    ref = torch.zeros(2, n, 1568, dtype=torch.bfloat16, device=DEV)
    out = torch.zeros_like(ref)
    job = eng._torso_job_sp(pt, ptl, rows, ref[0], ref[1])
    arr = np.asarray([job], dtype=np.int64)
    assert k.r2_torso_fwd_sp_multi(ptr(rp.frames), arr.ctypes.data, 1, 64, stream_handle()) == 0
    # qmode 1 with a stop word raised after ~1/3 of the frames: emulate with a pre-set counter
    eng.tq.zero_()
    eng.tq[0] = n // 3          # frames [0, n/3) "taken" by an earlier side launch ...
    job1 = eng._torso_job_sp(pt, ptl, rows, out[0], out[1], qmode=1)
    # ... which we compute here with a static job over the same rows
    job_s = eng._torso_job_sp(pt, ptl, rows[: n // 3], out[0, : n // 3], out[1, : n // 3])
    arr_s = np.asarray([job_s], dtype=np.int64)
    assert k.r2_torso_fwd_sp_multi(ptr(rp.frames), arr_s.ctypes.data, 1, 32, stream_handle()) == 0
    # a qmode-1 launch with the stop word already set takes nothing
    eng.tq[2] = 1
    arr1 = np.asarray([job1], dtype=np.int64)
    assert k.r2_torso_fwd_sp_multi(ptr(rp.frames), arr1.ctypes.data, 1, 32, stream_handle()) == 0
    torch.cuda.synchronize()
    assert int(eng.tq[0]) == n // 3
    # the remainder as a qmode-2 job beside a static online job (device-side deal)
    other = torch.zeros(2, 512, 1568, dtype=torch.bfloat16, device=DEV)
    other_ref = torch.zeros_like(other)
    jon = eng._torso_job_sp(eng.pk, eng.pk_lo, eng.rows[:512], other[0], other[1])
    jon_ref = eng._torso_job_sp(eng.pk, eng.pk_lo, eng.rows[:512], other_ref[0], other_ref[1])
    job2 = eng._torso_job_sp(pt, ptl, rows, out[0], out[1], qmode=2)
    arr2 = np.asarray([jon, job2], dtype=np.int64)
    assert k.r2_torso_fwd_sp_multi(ptr(rp.frames), arr2.ctypes.data, 2, 256, stream_handle()) == 0
    arr_r = np.asarray([jon_ref], dtype=np.int64)
    assert k.r2_torso_fwd_sp_multi(ptr(rp.frames), arr_r.ctypes.data, 1, 256, stream_handle()) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert torch.equal(other, other_ref)


@pytest.mark.parametrize("hoist", [False, True])
def test_fused_pack_tail_matches_separate_pack(hoist):
    """the weight repack riding on the priority tail (learner.fuse_pack_tail, plain
    step) against the separate pack_step launch, target sync every 2 steps: online and target
    packs, target master and step counter equal after every step (due and not-due steps).  With
    the hoisted step the pack is always its own launch (the tail runs beside the BPTT)."""
    rp0, a = _engine(hoist, B=16, interval=2, graph=True, **{"learner.fuse_pack_tail": True})
    rp1, b = _engine(hoist, B=16, interval=2, graph=True, **{"learner.fuse_pack_tail": False})
    a.capture(warmup=0)
    b.capture(warmup=0)
    for i in range(5):
        a.step()
        b.step()
        torch.cuda.synchronize()
        sa, sb = _state(rp0, a), _state(rp1, b)
        bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
        assert not bad, (i, bad)


@pytest.mark.parametrize("hoist", [False, True])
def test_folded_torso_reduce_matches_separate_launch(hoist):
    """Verdict r6 item 5: at world 1 the torso backward's slab reduction runs on the first
    workgroups of the optimizer launch (r2_rmsprop_pack_slab).  Weights, moments, packs, target
    and the gradient buffer equal the separate torso_grad_reduce launch's bitwise, every step."""
    rp0, a = _engine(hoist, B=16, interval=2, graph=True, **{"learner.fold_torso_reduce": True})
    rp1, b = _engine(hoist, B=16, interval=2, graph=True, **{"learner.fold_torso_reduce": False})
    assert a._fold_tq is not None and b._fold_tq is None
    a.capture(warmup=0)
    b.capture(warmup=0)
    for i in range(4):
        a.step()
        b.step()
        torch.cuda.synchronize()
        sa, sb = _state(rp0, a), _state(rp1, b)
        sa["grad"], sb["grad"] = a.grad, b.grad
        bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
        assert not bad, (i, bad)


def test_chunked_graph_matches_step_loop():
    """learner.graph_chunk: run_steps replays runs of m consecutive hoisted steps (even start, no
    target sync inside, previous step hoisted) as one graph.  Against the plain step loop, target
    sync every 7 steps (chunks around the sync steps fall back to single-step graphs): the same
    state bitwise after every run_steps call; at least two chunks replayed; error word 0."""
    rp0, plain = _engine(False, B=16, interval=7)
    rp1, ch = _engine(True, B=16, interval=7, **{"learner.graph_chunk": 4})
    plain.capture(warmup=0)
    ch.capture(warmup=0)
    assert ch._cgraph is not None
    for n in (1, 9, 4, 5, 8):
        for _ in range(n):
            plain.step()
        ch.run_steps(n)
        torch.cuda.synchronize()
        a, b = _state(rp0, plain), _state(rp1, ch)
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        assert not bad, (n, ch.steps_done, bad)
    assert ch.steps_done == plain.steps_done == 27
    assert getattr(ch, "chunks_run", 0) >= 2
    assert plain.error_word() == 0 and ch.error_word() == 0


def test_hoisted_step_without_fused_td_forks_after_td():
    """learner.td_fuse_head_bwd off: the TD launch is not the fused kernel that records the early
    fork and sets the done flag, so the side branch forks after TD as before -- still bitwise the
    plain step, error word 0."""
    kw = {"learner.td_fuse_head_bwd": False}
    rp0, plain = _engine(False, B=16, **kw)
    rp1, hoist = _engine(True, B=16, **kw)
    plain.capture(warmup=0)
    hoist.capture(warmup=0)
    for i in range(4):
        plain.step()
        hoist.step()
        torch.cuda.synchronize()
        a, b = _state(rp0, plain), _state(rp1, hoist)
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        assert not bad, (i, bad)
    assert plain.error_word() == 0 and hoist.error_word() == 0
