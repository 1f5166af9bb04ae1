"""Native host runtime: sum tree, shared-memory SPSC ring, fcntl lock, heartbeat table."""
import multiprocessing as mp
import os
import time
import uuid

import numpy as np
import pytest

from pytorch_r2d2_amd.runtime import FileLock, HeartbeatTable, ShmRing, SumTree


def test_sumtree_matches_numpy_and_samples_proportionally():
    rng = np.random.default_rng(0)
    cap = 5000
    t = SumTree(cap)
    leaves = np.zeros(cap)
    for _ in range(20):
        idx = rng.integers(0, cap, 300)
        val = rng.random(300) * (rng.random(300) < 0.7)
        t.set(idx, val)
        for i, v in zip(idx, val):   # last writer wins, like the tree
            leaves[i] = v
        assert t.total() == pytest.approx(leaves.sum(), rel=1e-9)
    n = 200_000
    s, p = t.sample(n, rng)
    assert np.all(leaves[s] > 0)
    assert np.allclose(p, leaves[s] / leaves.sum())
    bins = 10
    edges = np.linspace(0, cap, bins + 1).astype(int)
    exp = np.array([leaves[edges[i]:edges[i + 1]].sum() for i in range(bins)]) / leaves.sum() * n
    got = np.histogram(s, bins=edges)[0]
    assert np.max(np.abs(got - exp) / np.sqrt(exp)) < 5
    t2 = SumTree(cap)
    t2.rebuild(leaves)
    assert t2.total() == pytest.approx(t.total(), rel=1e-9)


def _producer(name, n):
    w = ShmRing(name, 1 << 14, create=False)
    for i in range(n):
        payload = (str(i) * (1 + i % 50)).encode()
        while not w.push(payload):
            time.sleep(0.0005)
    w.close(unlink=False)


def test_shm_ring_cross_process_ordering_and_wrap():
    name = f"/r2t_{uuid.uuid4().hex[:8]}"
    r = ShmRing(name, 1 << 14, create=True)
    n = 2000  # >> capacity: exercises wrap and back-pressure
    p = mp.get_context("spawn").Process(target=_producer, args=(name, n))
    p.start()
    got = []
    t0 = time.time()
    while len(got) < n and time.time() - t0 < 60:
        x = r.pop()
        if x is None:
            time.sleep(0.0002)
            continue
        got.append(x)
    p.join(30)
    r.close()
    assert p.exitcode == 0
    assert got == [(str(i) * (1 + i % 50)).encode() for i in range(n)]


def _try_lock(path, q):
    l = FileLock(path)
    q.put(l.acquire(blocking=False))
    l.close()


def test_file_lock_is_exclusive_across_processes(tmp_path):
    path = str(tmp_path / "data.pt")
    l = FileLock(path)
    assert l.acquire()
    q = mp.get_context("spawn").Queue()
    p = mp.get_context("spawn").Process(target=_try_lock, args=(path, q))
    p.start()
    assert q.get(timeout=60) is False
    p.join(30)
    l.release()
    p = mp.get_context("spawn").Process(target=_try_lock, args=(path, q))
    p.start()
    assert q.get(timeout=60) is True
    p.join(30)
    l.close()
    assert not os.path.exists(path)  # the lock never creates the data file


def test_heartbeat_table():
    name = f"/r2hb_{uuid.uuid4().hex[:8]}"
    h = HeartbeatTable(name, 3, create=True)
    assert h.age_s(1) == float("inf")
    h.beat(1, counter=7, status=2)
    r = h.read(1)
    assert r["counter"] == 7 and r["status"] == 2 and r["pid"] == os.getpid()
    assert h.age_s(1) < 1.0
    h.close()
