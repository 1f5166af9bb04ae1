"""Native run paths on the GPU: device-side trajectory ingest (files / shared-memory rings /
device records), CU-masked streams, the concurrent actor + learner driver (replay and weight
consistency invariants), and the CPU-actor -> HBM learner topology."""
import ctypes
import uuid

import numpy as np
import pytest
import torch

from pytorch_r2d2_amd.config import get_config
from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
from pytorch_r2d2_amd.ops._lib import kernels
from pytorch_r2d2_amd.replay.memory import ReplayMemory

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _small_cfg(**over):
    kw = {"replay.burn_in": 4, "replay.learn": 6, "replay.overlap": 5, "replay.n_step": 3,
          "learner.batch_size": 8}
    kw.update(over)
    return get_config("atari57", **kw)


def _record(n, seed, T=10, H=256):
    """An actor-style local replay of n rows with starts every 5 rows (window inside)."""
    rng = np.random.default_rng(seed)
    rm = ReplayMemory(n, 8, 3, (84, 84), H, 4, 4, obs_shape=(4, 84, 84))
    m = rm.memory
    m["state"][:] = rng.integers(0, 256, m["state"].shape, dtype=np.uint8)
    m["hs_cs"][:] = rng.normal(size=m["hs_cs"].shape)
    m["target_hs_cs"][:] = rng.normal(size=m["target_hs_cs"].shape)
    m["action"][:] = rng.integers(0, 6, m["action"].shape)
    m["reward"][:] = rng.normal(size=m["reward"].shape)
    m["done"][:] = (np.arange(n) >= n - 3)[:, None]
    m["priority"][:] = rng.random(n) + 0.1
    st = (np.arange(n) % 5 == 0) & (np.arange(n) <= n - T)
    m["is_seq_start"][:] = st
    m["sequence_priority"][:] = np.where(st, rng.random(n) + 0.5, 0)
    return m


def _check_replay_rows(rp, m, sub, head):
    n = m["state"].shape[0]
    rows = sub * rp.cap_e + (head + np.arange(n)) % rp.cap_e
    r = torch.as_tensor(rows, device=DEV)
    np.testing.assert_array_equal(rp.frames[r].cpu().numpy(), m["state"].reshape(n, -1))
    np.testing.assert_array_equal(rp.hs_cs[r].cpu().numpy(), m["hs_cs"])
    np.testing.assert_array_equal(rp.target_hs_cs[r].cpu().numpy(), m["target_hs_cs"])
    np.testing.assert_array_equal(rp.action[r].cpu().numpy(), m["action"].reshape(-1).astype(np.uint8))
    np.testing.assert_array_equal(rp.reward[r].cpu().numpy(), m["reward"].reshape(-1))
    np.testing.assert_array_equal(rp.done[r].cpu().numpy(), (m["done"].reshape(-1) > 0).astype(np.uint8))
    np.testing.assert_array_equal(rp.priority[r].cpu().numpy(), m["priority"])
    np.testing.assert_array_equal(rp.is_start[r].cpu().numpy(), m["is_seq_start"])
    np.testing.assert_array_equal(rp.tree[r].cpu().numpy(),
                                  (m["sequence_priority"] * m["is_seq_start"]).astype(np.float32))


def _tree_consistent(rp):
    leaves = rp.tree[: rp.capacity].double().sum().item()
    assert abs(rp.total_priority() - leaves) <= 1e-4 * max(1.0, leaves)
    assert int(rp.n_valid.item()) == int(rp.is_start.sum().item())


def test_ingest_memory_scatters_on_device_and_overwrites_old_starts():
    cfg = _small_cfg()
    rp = HBMReplay(cfg, DEV, capacity=2 * 300, n_subrings=2)
    m1, m2, m3 = _record(200, 1), _record(150, 2), _record(120, 3)
    assert rp.ingest_memory(m1, subring=0) == 200
    assert rp.ingest_memory(m2, subring=1) == 150
    torch.cuda.synchronize()
    _check_replay_rows(rp, m1, 0, 0)
    _check_replay_rows(rp, m2, 1, 0)
    _tree_consistent(rp)
    # sub-ring 0 wraps: rows 200..299 then 0..19 are overwritten; old starts there disappear
    assert rp.ingest_memory(m3, subring=0) == 120
    torch.cuda.synchronize()
    _check_replay_rows(rp, m3, 0, 200)
    assert int(rp.ihead[0].item()) == 20 and int(rp.rows_total_d.item()) == 470
    _tree_consistent(rp)
    assert int(rp.ingest_err.item()) == 0


def test_ingest_rejects_malformed_record():
    from pytorch_r2d2_amd.parallel.trajectory import pack_rows
    cfg = _small_cfg()
    rp = HBMReplay(cfg, DEV, capacity=256, n_subrings=1)
    m = _record(40, 5)
    m["hs_cs"] = m["hs_cs"][:, :100].copy()          # wrong state width
    buf = pack_rows(m)
    dev = torch.empty(buf.size + 64, dtype=torch.uint8, device=DEV)
    off = (-dev.data_ptr()) % 64
    dev[off: off + buf.size].copy_(torch.from_numpy(buf))
    rp.ingest_device_record(dev[off: off + buf.size], buf[:512], 0)
    torch.cuda.synchronize()
    assert int(rp.ingest_err.item()) & 1
    assert int(rp.n_valid.item()) == 0


def test_shm_ring_ingestor_dma_into_hbm():
    from pytorch_r2d2_amd.engine.ingest import HBMIngestor
    from pytorch_r2d2_amd.parallel.trajectory import ShmTrajectoryWriter
    cfg = _small_cfg()
    rp = HBMReplay(cfg, DEV, capacity=3 * 400, n_subrings=3)
    names = [f"/r2d2_gt_{uuid.uuid4().hex[:6]}_{i}" for i in range(3)]
    ing = HBMIngestor(rp, names, ring_bytes=64 << 20)
    try:
        writers = [ShmTrajectoryWriter(n, 64 << 20) for n in names]
        recs = {i: [_record(100 + 10 * i + j, 10 * i + j) for j in range(2)] for i in range(3)}
        for i, w in enumerate(writers):
            for m in recs[i]:
                w.push(m)
        total = 0
        for _ in range(10):
            total += ing.poll()
            ing._release_done(wait=True)
        torch.cuda.synchronize()
        assert total == sum(m["state"].shape[0] for ms in recs.values() for m in ms)
        for i in range(3):
            head = 0
            for m in recs[i]:
                _check_replay_rows(rp, m, i, head)
                head += m["state"].shape[0]
        _tree_consistent(rp)
        assert all(ws.ring.used() >= 0 for ws in writers)
        assert all(r.ring.front() is None for r in ing.readers)
        print("zero-copy registered rings:", [b is not None for b in ing.registered])
    finally:
        ing.close()


def test_ingest_poll_dirty_budget_spans_all_records():
    """One poll ingests one record per ring and repairs the tree once: the records' dirty
    entries share one list.  4 rings x 40 rows that are all sequence starts = 160 entries on a
    128-entry list -- each record alone fits, together they would overflow (entries past the list
    are dropped and the tree keeps stale sums); the poll must fall back to a full rebuild."""
    from pytorch_r2d2_amd.engine.ingest import HBMIngestor
    from pytorch_r2d2_amd.parallel.trajectory import ShmTrajectoryWriter
    cfg = _small_cfg()
    rp = HBMReplay(cfg, DEV, capacity=4 * 200, n_subrings=4)
    rp.max_dirty = 128
    rp.dirty = rp.dirty[:128]
    names = [f"/r2d2_gd_{uuid.uuid4().hex[:6]}_{i}" for i in range(4)]
    ing = HBMIngestor(rp, names, ring_bytes=16 << 20)
    try:
        writers = [ShmTrajectoryWriter(n, 16 << 20) for n in names]
        for i, w in enumerate(writers):
            m = _record(40, 50 + i)
            m["is_seq_start"][:] = 1
            m["sequence_priority"][:] = np.random.default_rng(i).random(40) + 0.5
            w.push(m)
        assert ing.poll() == 160
        ing._release_done(wait=True)
        torch.cuda.synchronize()
        assert int(rp.n_valid.item()) == 160
        _tree_consistent(rp)
    finally:
        ing.close()


def test_ingestor_drops_malformed_records_uncounted():
    """A record whose header does not match the schema, or whose n exceeds its payload, is
    dropped on the host before any DMA (not counted as ingested); a forged header that reaches
    the device kernel is rejected there without advancing the write head or the row counter."""
    from pytorch_r2d2_amd.engine.ingest import HBMIngestor
    from pytorch_r2d2_amd.parallel.trajectory import ShmTrajectoryWriter, pack_rows
    cfg = _small_cfg()
    rp = HBMReplay(cfg, DEV, capacity=2 * 200, n_subrings=2)
    names = [f"/r2d2_gm_{uuid.uuid4().hex[:6]}_{i}" for i in range(2)]
    ing = HBMIngestor(rp, names, ring_bytes=16 << 20)
    try:
        w = [ShmTrajectoryWriter(n, 16 << 20) for n in names]
        bad = _record(30, 7)
        bad["hs_cs"] = bad["hs_cs"][:, :100].copy()
        w[0].push(bad)
        good = _record(30, 8)
        w[1].push(good)
        assert ing.poll() == 30
        ing._release_done(wait=True)
        torch.cuda.synchronize()
        assert ing.rejected == 1 and ing.records == 1 and ing.rows == 30
        _check_replay_rows(rp, good, 1, 0)
        ing.check_errors()
    finally:
        ing.close()
    # device side: n in the header larger than the fields hold
    buf = pack_rows(_record(20, 9))
    buf[8:16] = np.asarray([5000], dtype=np.int64).view(np.uint8)
    dev = torch.empty(buf.size + 64, dtype=torch.uint8, device=DEV)
    off = (-dev.data_ptr()) % 64
    dev[off: off + buf.size].copy_(torch.from_numpy(buf))
    head0, tot0 = rp.ihead.clone(), rp.rows_total_d.clone()
    rp.ingest_device_record(dev[off: off + buf.size], None, 0)
    torch.cuda.synchronize()
    assert int(rp.ingest_err.item()) & 1
    assert torch.equal(rp.ihead, head0) and torch.equal(rp.rows_total_d, tot0)


def test_cu_masked_streams_partition_the_chip():
    from pytorch_r2d2_amd.parallel.placement import split_chip
    sa, sl, na, nl, per_l = split_chip(DEV, 4)
    want = {"actor": [4] * 8, "learner": [28] * 8}
    try:
        assert na == 32 and nl == torch.cuda.get_device_properties(0).multi_processor_count - 32
        assert per_l == want["learner"]
        k = kernels()
        seen = {}
        for name, s in (("actor", sa), ("learner", sl)):
            out = torch.zeros(2 * 2048, dtype=torch.int32, device=DEV)
            # eager launch and the same launch replayed as a graph on the masked stream
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            with torch.cuda.graph(g, stream=side):
                assert k.r2_cu_probe(ctypes.c_void_p(out.data_ptr()), 2048, 2,
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
            with torch.cuda.stream(s.stream):
                g.replay()
            torch.cuda.synchronize()
            v = out.view(-1, 2).cpu().numpy()
            cus = {(int(x), (int(h) >> 8) & 15, (int(h) >> 13) & 7) for x, h in v}
            seen[name] = cus
            per = np.bincount([c[0] for c in cus], minlength=8)
            assert list(per) == want[name], (name, per)
        assert not (seen["actor"] & seen["learner"])
    finally:
        sa.close()
        sl.close()


def _concurrent_setup(E=16, cap_e=512, M=2, masked=True, **over):
    from pytorch_r2d2_amd.actor_batched import BatchedActor, engine_weights
    from pytorch_r2d2_amd.engine.concurrent import ConcurrentDriver
    from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
    from pytorch_r2d2_amd.envs.synthetic import VecSyntheticAtari
    from pytorch_r2d2_amd.parallel.placement import split_chip
    cfg = _small_cfg(**{"learner.publish_interval": 5, "actor.envs_per_actor": E,
                        "learner.target_update_interval": 7, **over})
    sa = sl = None
    na, nl = 256, None
    if masked:
        sa, sl, na, nl, _ = split_chip(DEV, 4)
    rp = HBMReplay(cfg, DEV, capacity=E * cap_e, n_subrings=E)
    eng = LearnerEngine(cfg, rp, DEV, n_cus=nl)
    env = VecSyntheticAtari(E, DEV, seed=3, episode_len=37, n_actions=cfg.model.n_actions)
    on, tg = engine_weights(eng)
    actor = BatchedActor(cfg, rp, env, on, tg, seed=1)
    while int(rp.n_valid.item()) < 4 * cfg.learner.batch_size:
        actor.step()
    eng.capture(warmup=1)
    actor.n_workers = na
    drv = ConcurrentDriver(eng, actor, steps_per_round=M,
                           actor_stream=sa.stream if sa else None,
                           learner_stream=sl.stream if sl else None)
    return cfg, rp, eng, actor, drv, (sa, sl)


@pytest.mark.parametrize("masked", [True, False], ids=["cu_masked", "shared_chip"])
def test_concurrent_driver_never_samples_rows_being_written(masked):
    cfg, rp, eng, actor, drv, streams = _concurrent_setup(masked=masked)
    B, Tn = cfg.learner.batch_size, cfg.replay.seq_len + cfg.replay.n_step
    R = 120
    hist = torch.zeros(R, B, dtype=torch.int32, device=DEV)

    def log_starts(i):
        if i < R:
            hist[i].copy_(eng.starts)
    drv.on_learner_step = log_starts
    drv.run(R)
    drv.finish()
    drv.check_errors()
    starts = hist.cpu().numpy()
    done = rp.done.cpu().numpy()
    cap_e, M, T = rp.cap_e, drv.M, cfg.replay.seq_len
    assert drv.rounds * M + drv.heads[0] < cap_e          # no wrap: rows keep their round's data
    n_ext = 0
    for r in range(R):
        written = {(drv.heads[r] + j) % cap_e for j in range(M)}
        for s in starts[r]:
            off, base = s % cap_e, s - s % cap_e
            window = {(off + t) % cap_e for t in range(T)}
            assert not (window & written), (r, s)
            # the n bootstrap frames past the window may be the next episode's first rows (being
            # written): only for a final start, whose last learning row is terminal (masked)
            ext = {(off + t) % cap_e for t in range(T, Tn)}
            if ext & written:
                n_ext += 1
                assert done[base + (off + T - 1) % cap_e] == 1, (r, s)
    print("samples whose masked bootstrap frames were being written:", n_ext)
    # weights: published every 5 learner steps; the actor's copy is the last published master
    assert drv.version == R // 5
    torch.testing.assert_close(drv.w_on.flat, drv.stage_on, rtol=0, atol=0)
    assert drv.w_on.version == drv.version
    # replay bookkeeping stayed consistent while both roles mutated it
    _tree_consistent(rp)
    for s in streams:
        if s is not None:
            s.close()


def test_run_native_concurrent_and_serial_train():
    from pytorch_r2d2_amd.runner import run_native
    cfg = _small_cfg(**{"actor.envs_per_actor": 32, "learner.publish_interval": 10})
    outs = {}
    for mode, conc, k in (("serial", False, 0), ("masked", True, 4), ("shared", True, 0)):
        out = run_native(cfg, steps=60, actor_steps_per_update=2, warmup_rows=32 * 120,
                         capacity=32 * 600, log_every=30, concurrent=conc, actor_cus_per_xcd=k,
                         check_every=20)
        assert all(np.isfinite(out["losses"]))
        outs[mode] = out
        print(mode, {k: out[k] for k in ("learner_steps_per_s", "env_steps_per_s", "learner_cus")})
    assert outs["masked"]["learner_cus"] < outs["serial"]["learner_cus"] == outs["shared"]["learner_cus"]
    assert outs["masked"]["weights_version"] == outs["shared"]["weights_version"] == 6


@pytest.mark.slow
def test_cpu_actor_processes_feed_the_hbm_learner(tmp_path):
    from pytorch_r2d2_amd.runner import run_native_cpu_actors
    cfg = get_config("pong", **{"replay.burn_in": 4, "replay.learn": 6, "replay.overlap": 5,
                                "env.episode_len": 40, "actor.memory_save_interval": 1,
                                "actor.net_load_interval": 1, "learner.publish_interval": 5})
    out = run_native_cpu_actors(cfg, 2, steps=20, warmup_rows=150, capacity=2 * 4096,
                                log_every=10, timeout_s=240, stall_timeout_s=120)
    assert out["steps"] == 20, out
    assert out["ingested_rows"] >= 150 and out["records"] >= 2
    print({k: out[k] for k in ("ingest_rows_per_s", "learner_steps_per_s", "zero_copy",
                               "ingested_rows")})


def _traj_worker(rank, world, port, outdir):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    from pytorch_r2d2_amd.parallel.channel import LinkReceiver, LinkSender
    from pytorch_r2d2_amd.parallel.trajectory import header_bytes, pack_rows
    dist.init_process_group("gloo")
    recs = [torch.from_numpy(pack_rows(_record(90 + j, 40 + j))) for j in range(2)]
    nb = max(r.numel() for r in recs)
    if rank == 0:
        tx = LinkSender("traj/0", 1, nb, 2, "cpu")
        for r in recs:
            b = tx.acquire()
            b.zero_()
            b[: r.numel()].copy_(r)
            tx.send()
        tx.flush()
        tx.close()
    else:
        rp = HBMReplay(_small_cfg(), DEV, capacity=2 * 256, n_subrings=2)
        got = []

        def ingest(i, buf):
            d = buf.to(DEV)
            got.append(rp.ingest_device_record(d, buf[: header_bytes()].numpy(), subring=1))

        rx = LinkReceiver(["traj/0"], [0], nb, "cpu", ingest)
        rx.wait_closed()
        torch.cuda.synchronize()
        _check_replay_rows(rp, _record(90, 40), 1, 0)
        _check_replay_rows(rp, _record(91, 41), 1, 90)
        _tree_consistent(rp)
        torch.save({"got": got}, os.path.join(outdir, "traj.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_trajectory_link_ingests_into_hbm_replay(tmp_path):
    """Host-packed records over an asynchronous link (parallel/channel.py, gloo) into a device
    record buffer and the HBM replay's sub-ring 1 (the ingest kernel): rows bit-identical, the
    sum tree consistent."""
    import os
    import socket
    import torch.multiprocessing as tmp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    tmp.spawn(_traj_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    assert torch.load(os.path.join(tmp_path, "traj.pt"), weights_only=True)["got"] == [90, 91]


@pytest.mark.parametrize("fused", [False, True], ids=["td_kernel", "td_duel"])
def test_td_row_priorities_last_write_wins(fused):
    """Overlapping / duplicate sampled sequences: the row priority written is the one of the LAST
    (t, b) in row-major order, as numpy resolves the reference's duplicate-index assignment
    (learner.py:101-103); deterministic across runs."""
    from pytorch_r2d2_amd.ops._lib import ptr
    k = kernels()
    g = torch.Generator(device="cpu").manual_seed(0)
    Tl, B, A, Lb, cap_e, HD = 6, 8, 6, 2, 64, 64
    starts = torch.tensor([3, 5, 3, 64 + 10, 60, 7, 5, 62], dtype=torch.int32)   # dups, overlaps, wrap
    q = [torch.randn(Tl * B, A, generator=g) for _ in range(3)]
    cap = 2 * cap_e
    action = torch.randint(0, A, (cap,), generator=g).to(torch.uint8)
    reward = torch.randn(cap, generator=g)
    done = torch.zeros(cap, dtype=torch.uint8)
    d = lambda t: t.to(DEV).contiguous()  # noqa: E731
    qs, qa, qt = (d(x) for x in q)
    st, act, rew, dn = d(starts), d(action), d(reward), d(done)
    outs = []
    for rep in range(2):
        prio = torch.full((cap,), -1.0, device=DEV)
        dq = torch.zeros(Tl * B, A, device=DEV)
        loss, tdabs = torch.zeros(1, device=DEV), torch.zeros(Tl * B, device=DEV)
        part, ticket = torch.zeros(4096, device=DEV), torch.zeros(1, dtype=torch.int32, device=DEV)
        args = (ptr(qs), ptr(qa), ptr(qt), ptr(st), 0, ptr(act), ptr(rew), ptr(dn), ptr(dq), ptr(loss),
                ptr(tdabs), ptr(prio), 0, 0, Tl, B, A, Lb, cap_e, 0.99, 0, 1e-3, 0.9, 1e-6, 0.0,
                ptr(part), ptr(ticket))
        if fused:
            zr = torch.randn(Tl * B, 2 * HD, generator=g).to(torch.bfloat16).to(DEV)
            w2 = torch.randn(1 + A, HD, generator=g).to(DEV)
            dz = torch.zeros(Tl * B, 2 * HD, dtype=torch.bfloat16, device=DEV)
            dva = torch.zeros(Tl * B, 1 + A, device=DEV)
            assert k.r2_td_duel(*args, ptr(zr), ptr(w2), ptr(dz), ptr(dva), HD, 0, 0,
                                torch.cuda.current_stream().cuda_stream) == 0
        else:
            assert k.r2_td_loss(*args, 0, torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        outs.append(prio.cpu())
        ad = tdabs.cpu().numpy().reshape(Tl, B)
    # numpy reference: index[burn_in:].reshape(-1) = prio.reshape(-1), last write wins
    ref = np.full(cap, -1.0, dtype=np.float32)
    s = starts.numpy().astype(np.int64)
    rows = (s - s % cap_e)[None, :] + (s % cap_e + Lb + np.arange(Tl)[:, None]) % cap_e   # (Tl, B)
    ref[rows.reshape(-1)] = ((ad + 1e-6) ** 0.9).reshape(-1)
    np.testing.assert_allclose(outs[0].numpy(), ref, rtol=1e-6)
    assert torch.equal(outs[0], outs[1])


def test_actor_rank_block_pack_and_lagged_ingest():
    """Split topology data path without the network: an actor group's newest FINAL rows (K per env
    per round, n steps behind the write head, each row shipped once) packed on the device
    (pack_rows_kernel) with the start column lagged by W - 1 rows, and scattered env-major into a
    learner replay (ingest_rows_kernel, start_lag): every row bit-identical to the actor's stream
    row n earlier, every start set exactly when the last row of its window arrives, a row's own
    start cleared until then, the tree consistent."""
    import ctypes as C
    from pytorch_r2d2_amd.actor_batched import BatchedActor, PackedWeights
    from pytorch_r2d2_amd.engine.ingest import ingest_args
    from pytorch_r2d2_amd.engine.layout import ParamLayout
    from pytorch_r2d2_amd.envs.synthetic import VecSyntheticAtari
    from pytorch_r2d2_amd.models import QNet
    from pytorch_r2d2_amd.ops._lib import ptr, stream_handle
    from pytorch_r2d2_amd.parallel.actor_ranks import TrajectoryPusher
    cfg = _small_cfg()
    E, K = 4, 16
    n = cfg.replay.n_step
    W = cfg.replay.seq_len + n
    lag = W - 1
    act_rp = HBMReplay(cfg, DEV, capacity=E * 128, n_subrings=E)
    L = ParamLayout(cfg.model, cfg.env)
    w = PackedWeights(L, DEV)
    torch.manual_seed(0)
    w.load(QNet("cpu", cfg.model, cfg.env).state_dict())
    env = VecSyntheticAtari(E, DEV, seed=9, episode_len=23)
    actor = BatchedActor(cfg, act_rp, env, w, w, seed=2)
    push = TrajectoryPusher(act_rp, K, dst=0, link=False)
    raw = torch.zeros(push.nbytes + 64, dtype=torch.uint8, device=DEV)
    off = (-raw.data_ptr()) % 64
    rec = raw[off: off + push.nbytes]
    rec[: push.hdr.numel()].copy_(push.hdr)
    lrn = HBMReplay(cfg, DEV, capacity=E * 300, n_subrings=E)
    ca, cl = act_rp.cap_e, lrn.cap_e
    er = torch.arange(E, device=DEV)[:, None]
    jr = torch.arange(K, device=DEV)[None, :]
    shipped_starts = 0
    for c in range(12):
        for _ in range(K):
            actor.step()
        push.pack(c, rec)
        a = ingest_args(lrn, ptr(rec), push.nbytes, 0, True, rows_per_sub=K, start_lag=lag)
        assert kernels().r2_ingest_record(C.byref(a), C.c_void_p(stream_handle())) == 0
        lrn.repair_after_ingest()
        torch.cuda.synchronize()
        a_rows = (er * ca + (c * K + jr - n) % ca).reshape(-1)
        l_rows = (er * cl + (c * K + jr) % cl).reshape(-1)
        for name in ("frames", "hs_cs", "target_hs_cs", "action", "reward", "done", "priority"):
            assert torch.equal(getattr(lrn, name)[l_rows], getattr(act_rp, name)[a_rows]), (c, name)
        # starts: this record marks learner positions cK + j - lag (actor stream rows n earlier);
        # stream rows < 0 never start; the record's own rows j >= K - lag (windows not complete
        # yet) stay non-starts
        s_l = (er * cl + (c * K + jr - lag) % cl).reshape(-1)
        s_a = (er * ca + (c * K + jr - lag - n) % ca).reshape(-1)
        keep = ((c * K + jr - lag - n) >= 0).expand(E, K).reshape(-1)
        exp = act_rp.is_start[s_a].bool() & keep
        assert torch.equal(lrn.is_start[s_l].bool(), exp), c
        assert torch.equal(lrn.tree[s_l], torch.where(exp, act_rp.tree[s_a], 0.0)), c
        own = (er * cl + (c * K + torch.arange(max(0, K - lag), K, device=DEV)[None, :]) % cl).reshape(-1)
        assert not lrn.is_start[own].bool().any(), c
        shipped_starts += int(exp.sum())
        assert int(lrn.ihead[0]) == (c + 1) * K % cl
    _tree_consistent(lrn)
    assert shipped_starts > 20 and int(lrn.ingest_err.item()) == 0
    # a record that addresses sub-rings past the replay's is rejected (error word), not written
    a = ingest_args(lrn, ptr(rec), push.nbytes, 1, True, rows_per_sub=K, start_lag=lag)
    head = lrn.ihead.clone()
    assert kernels().r2_ingest_record(C.byref(a), C.c_void_p(stream_handle())) == 0
    torch.cuda.synchronize()
    assert int(lrn.ingest_err.item()) != 0 and torch.equal(lrn.ihead, head)


def _split_worker(rank, world, port, outdir):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    from pytorch_r2d2_amd.runner import run_split
    cfg = _small_cfg(**{"actor.envs_per_actor": 8, "dist.push_rows": 16, "dist.publish_steps": 4,
                        "env.episode_len": 30})
    out = run_split(cfg, rounds=16, actor_ranks=world - 1, capacity=8 * 600, backend="gloo",
                    log_every=0, learner_steps=12)
    keep = {k: v for k, v in out.items() if isinstance(v, (int, float, str)) or v is None}
    if out["role"] == "learner":
        keep["master"] = out["engine"].master.detach().cpu()
    torch.save(keep, os.path.join(outdir, f"split{rank}.pt"))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def test_split_topology_actor_rank_feeds_learner_rank(tmp_path):
    """run_split with 1 learner rank + 1 actor rank sharing this GPU (gloo staging): 16 rounds of
    device-packed blocks over the asynchronous link -> learner ingest -> 12 training steps,
    weights published every 4 learner steps; every record arrives, nothing is lost."""
    import socket
    import torch.multiprocessing as tmp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    tmp.spawn(_split_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    lr = torch.load(tmp_path / "split0.pt", weights_only=True)
    ac = torch.load(tmp_path / "split1.pt", weights_only=True)
    assert lr["role"] == "learner" and ac["role"] == "actor"
    assert ac["windows"] == 16 and lr["records"] == 16
    assert lr["rows_ingested"] == 16 * 8 * 16            # rounds x E x K: each row once
    assert lr["learner_steps"] == 12 and lr["n_valid"] > 0 and lr["ingest_err"] == 0
    assert ac["weights_version"] == lr["weights_version"] >= 2
    assert torch.isfinite(lr["master"]).all()
