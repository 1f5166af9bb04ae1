"""Native transports on the CPU: aligned trajectory records, zero-copy ring consumption, the
seqlock weight slot (never torn across processes), the shared-memory weight writer / reader,
CU-mask words, and failure handling wired into the real roles (compat topology)."""
import multiprocessing as mp
import os
import time
import uuid

import numpy as np
import pytest
import torch

from pytorch_r2d2_amd.config import get_config
from pytorch_r2d2_amd.parallel.trajectory import (ALIGN, ORDER, header_bytes, pack_rows,
                                                  record_layout, unpack_rows)
from pytorch_r2d2_amd.replay.memory import ReplayMemory
from pytorch_r2d2_amd.runtime import ShmRing, ShmSlot


def _mem(n=37, seed=0, shape=(4, 84, 84), H=256):
    rng = np.random.default_rng(seed)
    rm = ReplayMemory(n, 8, 3, shape[1:], H, 4, 4, obs_shape=shape)
    m = rm.memory
    m["state"][:] = rng.integers(0, 256, m["state"].shape, dtype=np.uint8)
    m["hs_cs"][:] = rng.normal(size=m["hs_cs"].shape)
    m["target_hs_cs"][:] = rng.normal(size=m["target_hs_cs"].shape)
    m["action"][:] = rng.integers(0, 6, m["action"].shape)
    m["reward"][:] = rng.normal(size=m["reward"].shape)
    m["done"][:] = rng.random(m["done"].shape) < 0.1
    m["priority"][:] = rng.random(n)
    m["is_seq_start"][:] = rng.random(n) < 0.2
    m["sequence_priority"][:] = rng.random(n) * m["is_seq_start"]
    return m


def test_record_roundtrip_and_alignment():
    m = _mem()
    buf = pack_rows(m)
    n, fields = record_layout(buf)
    assert n == 37 and list(fields) == list(ORDER)
    assert header_bytes() % ALIGN == 0
    for name, (code, per_row, nbytes, off) in fields.items():
        assert off % ALIGN == 0, name
        assert nbytes == m[name].nbytes
    back = unpack_rows(buf, state_shape=(4, 84, 84))
    for k in ORDER:
        np.testing.assert_array_equal(np.asarray(back[k]).reshape(m[k].shape), m[k])


def test_ring_front_is_zero_copy_and_release_advances():
    name = f"/r2d2_t_{uuid.uuid4().hex[:8]}"
    ring = ShmRing(name, 1 << 20, create=True)
    try:
        assert ring.front() is None
        a, b = b"x" * 1000, b"y" * 3000
        assert ring.push(a) and ring.push(b)
        addr, n = ring.front()
        assert n == 1000
        import ctypes
        assert ctypes.string_at(addr, n) == a
        assert ring.front() == (addr, n)          # peek does not consume
        ring.release()
        addr2, n2 = ring.front()
        assert n2 == 3000 and ctypes.string_at(addr2, n2) == b
        ring.release()
        assert ring.front() is None and ring.used() == 0
        base, size = ring.mapping()
        assert base <= addr < base + size
    finally:
        ring.close(unlink=True)


def _slot_writer(name, n, stop_after):
    s = ShmSlot(name, n * 4, create=False)
    t0 = time.time()
    v = 0
    while time.time() - t0 < stop_after:
        v += 1
        s.write(np.full(n, v, dtype=np.float32), v)
    s.close(unlink=False)


def test_seqlock_slot_is_never_torn_across_processes():
    n = 1 << 18                    # 1 MB blob: a torn read would mix two versions
    name = f"/r2d2_s_{uuid.uuid4().hex[:8]}"
    slot = ShmSlot(name, n * 4, create=True)
    try:
        assert slot.read(np.zeros(n, np.float32)) is None       # nothing published yet
        ctx = mp.get_context("spawn")
        p = ctx.Process(target=_slot_writer, args=(name, n, 3.0))
        p.start()
        out = np.zeros(n, np.float32)
        have, reads = -1, 0
        t0 = time.time()
        while time.time() - t0 < 20 and (p.is_alive() or reads == 0):
            v = slot.read(out, have)
            if v is not None:
                assert v > have
                assert out[0] == v and np.all(out == out[0]), "torn read"
                have, reads = v, reads + 1
        p.join(10)
        assert reads > 3
        assert slot.read(out, have) is None       # nothing newer than what we hold
    finally:
        slot.close(unlink=True)


def test_shm_weights_writer_reader_roundtrip():
    from pytorch_r2d2_amd.engine.layout import ParamLayout
    from pytorch_r2d2_amd.models import QNet
    from pytorch_r2d2_amd.parallel.weights import ShmWeightsReader, ShmWeightsWriter
    cfg = get_config("reference")
    L = ParamLayout(cfg.model, cfg.env)
    torch.manual_seed(0)
    on, tg = QNet("cpu", cfg.model, cfg.env), QNet("cpu", cfg.model, cfg.env)
    f_on, f_tg = L.from_module(on, "cpu"), L.from_module(tg, "cpu")
    name = f"/r2d2_w_{uuid.uuid4().hex[:8]}"
    w = ShmWeightsWriter(name, L.padded, "cpu")
    try:
        r = ShmWeightsReader(name, cfg)
        assert r.fetch() is None
        w.publish(f_on, f_tg, 3)
        sd_on, sd_tg, v = r.fetch(-1)
        assert v == 3 and r.fetch(3) is None
        for k, t in on.state_dict().items():
            torch.testing.assert_close(sd_on[k], t, rtol=0, atol=0)
        for k, t in tg.state_dict().items():
            torch.testing.assert_close(sd_tg[k], t, rtol=0, atol=0)
        # an actor reading through the slot loads exactly the published nets
        from pytorch_r2d2_amd.actor import Actor
        a = Actor(0, 1, None, "cpu", cfg=cfg)
        a.weights_reader = r
        w.publish(f_tg, f_on, 4)      # swapped, to see it land
        assert a.load_model() and a.weights_version == 4
        for k, t in tg.state_dict().items():
            torch.testing.assert_close(a.net.state_dict()[k], t, rtol=0, atol=0)
    finally:
        w.close()


def test_cu_mask_words_split_every_xcd():
    from pytorch_r2d2_amd.parallel.placement import cu_mask_words
    a = cu_mask_words(256, 4, True)
    b = cu_mask_words(256, 4, False)
    assert len(a) == 8 and a[0] == 0xFFFFFFFF and all(x == 0 for x in a[1:])
    assert b[0] == 0 and all(x == 0xFFFFFFFF for x in b[1:])
    bits = lambda ws: {i for i, w in enumerate(ws) for i in [i * 32 + j for j in range(32) if w >> j & 1]}  # noqa: E731
    sa, sb = bits(a), bits(b)
    assert not (sa & sb) and len(sa | sb) == 256
    # bit i -> XCD i % 8 (measured): both sets hold the same count of every XCD
    for x in range(8):
        assert sum(1 for i in sa if i % 8 == x) == 4
        assert sum(1 for i in sb if i % 8 == x) == 28
    with pytest.raises(ValueError):
        cu_mask_words(256, 32, True)


def _actor_push_proc(ring_name, n_records, rows, seed):
    from pytorch_r2d2_amd.parallel.trajectory import ShmTrajectoryWriter
    w = ShmTrajectoryWriter(ring_name, 8 << 20)
    for i in range(n_records):
        w.push(_mem(rows, seed * 100 + i, shape=(4, 8, 8), H=16))


def test_shm_trajectory_ring_delivers_records_in_order_across_processes():
    from pytorch_r2d2_amd.parallel.trajectory import ShmTrajectoryReader
    name = f"/r2d2_r_{uuid.uuid4().hex[:8]}"
    rd = ShmTrajectoryReader(name, 8 << 20, state_shape=(4, 8, 8))
    try:
        ctx = mp.get_context("spawn")
        p = ctx.Process(target=_actor_push_proc, args=(name, 12, 50, 7))
        p.start()
        got = []
        t0 = time.time()
        while len(got) < 12 and time.time() - t0 < 60:
            got += rd.poll()
            time.sleep(0.005)
        p.join(10)
        assert len(got) == 12
        for i, g in enumerate(got):
            ref = _mem(50, 700 + i, shape=(4, 8, 8), H=16)
            np.testing.assert_array_equal(g["state"], ref["state"])
            np.testing.assert_array_equal(g["hs_cs"], ref["hs_cs"])
    finally:
        rd.close()


@pytest.mark.slow
def test_compat_roles_heartbeat_restart_crashed_actor_while_learner_trains(monkeypatch, tmp_path):
    """The REAL roles (actor_process / learner_process) beat and honour fault hooks: actor 0
    crashes at step 40 and is restarted as a fresh process, the learner keeps training to its
    step budget."""
    from pytorch_r2d2_amd.runner import run_compat
    monkeypatch.setenv("R2D2_FAULTS", "actor:0:crash_at=40")
    cfg = get_config("cartpole", **{"learner.initial_exploration": 100, "learner.batch_size": 4,
                                    "replay.burn_in": 4, "replay.learn": 4, "replay.overlap": 4,
                                    "actor.memory_save_interval": 1, "learner.ingest_interval": 1,
                                    "learner.checkpoint_interval": 100000,
                                    "learner.save_dir": str(tmp_path / "save")})
    rep = run_compat(cfg, 2, steps=30, memory_path=str(tmp_path / "mem"), timeout_s=150,
                     stall_timeout_s=30.0)
    assert rep["actor0"]["restarts"] >= 1 and 17 in rep["actor0"]["exitcodes"]
    assert rep["learner"]["exitcodes"] == [0], rep


@pytest.mark.slow
def test_compat_learner_hang_is_detected(monkeypatch, tmp_path):
    from pytorch_r2d2_amd.runner import run_compat
    monkeypatch.setenv("R2D2_FAULTS", "learner:0:hang_at=0")
    cfg = get_config("cartpole", **{"learner.save_dir": str(tmp_path / "save")})
    t0 = time.time()
    rep = run_compat(cfg, 1, steps=10, memory_path=str(tmp_path / "mem"), timeout_s=120,
                     learner_stall_timeout_s=3.0)
    assert rep["learner"]["stalls"] == 1
    assert time.time() - t0 < 100
