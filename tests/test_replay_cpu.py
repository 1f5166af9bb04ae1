"""Golden semantic tests for the replay layer: n-step emission, sequence priority
(eta-mix, wraparound, neighbour refresh), schema, sampling, file transport."""
import os

import numpy as np
import pytest
import torch

from pytorch_r2d2_amd.replay import NStepMemory, ReplayMemory


def _fill(nm, n):
    for k in range(n):
        nm.add(q_value=k, state=f"s{k}", hs=0, cs=0, target_hs=0, target_cs=0, action=0,
               reward=float(k + 1), stack_count=1)


def test_nstep_legacy_reproduces_q3_first_transition_lost():
    nm = NStepMemory(3, 0.5, legacy=True)
    _fill(nm, 4)
    out = nm.get()
    assert out[1] == "s1"  # replay_memory.py:17-25 maxlen eviction drops s0 (Q3)


def test_nstep_legacy_reproduces_q4_identical_tail_returns():
    g = 0.5
    nm = NStepMemory(3, g, legacy=True)
    _fill(nm, 5)  # deque holds s2,s3,s4 with rewards 3,4,5
    rets = [nm.get()[7] for _ in range(3)]
    expect = 3 + g * 4 + g * g * 5
    assert rets == [pytest.approx(expect)] * 3


def test_nstep_fixed_returns_and_tail():
    g = 0.5
    nm = NStepMemory(3, g)
    _fill(nm, 5)
    outs = [nm.get() for _ in range(5)]
    assert [o[1] for o in outs] == ["s0", "s1", "s2", "s3", "s4"]
    r = [1, 2, 3, 4, 5]
    exp = [r[k] + g * (r[k + 1] if k + 1 < 5 else 0) + g * g * (r[k + 2] if k + 2 < 5 else 0) for k in range(5)]
    assert [o[7] for o in outs] == pytest.approx(exp)
    assert nm.size == 0


def _mem(cap=100, legacy=False, **kw):
    return ReplayMemory(cap, 4, 3, legacy=legacy, **kw)


def test_schema_matches_reference():
    m = _mem(10)
    spec = {"state": ((10, 4, 84, 84), np.uint8), "hs_cs": ((10, 512), np.float32),
            "target_hs_cs": ((10, 512), np.float32), "action": ((10, 1), np.int8),
            "reward": ((10, 1), np.float32), "done": ((10, 1), np.float32),
            "stack_count": ((10,), np.int8), "priority": ((10,), np.float32),
            "sequence_priority": ((10,), np.float32), "is_seq_start": ((10,), np.uint8)}
    for k, (shape, dt) in spec.items():
        assert m.memory[k].shape == shape and m.memory[k].dtype == dt, k
    row_bytes = sum(v.nbytes for v in m.memory.values()) // 10
    assert row_bytes == 32339


def test_state_quantisation_lossless():
    m = _mem(4)
    x = np.arange(256, dtype=np.uint8).repeat(111)[: 4 * 84 * 84].reshape(4, 84, 84)
    m.add(x.astype(np.float32) / 255.0, np.zeros(256), np.zeros(256), np.zeros(256), np.zeros(256),
          1, 0.5, False, 1, 0.3)
    assert np.array_equal(m.memory["state"][0], x)


def test_sequence_priority_wraparound_q9():
    for legacy, expect in ((True, 1.0), (False, 0.9 * 50 + 0.1 * (5 * 1 + 15 * 50) / 20)):
        m = _mem(100, legacy=legacy, burn_in=10, learning=10)
        m.memory["priority"][95:100] = 1.0
        m.memory["priority"][0:15] = 50.0
        m.update_sequence_priority([95])
        assert m.memory["sequence_priority"][95] == pytest.approx(expect)


def test_neighbour_refresh_q8():
    def changed(legacy):
        m = _mem(100, legacy=legacy, burn_in=10, learning=10)
        m.memory["is_seq_start"][[30, 40, 50, 60, 70]] = 1
        m.memory["priority"][:] = np.arange(100, dtype=np.float32)
        before = m.memory["sequence_priority"].copy()
        m.update_sequence_priority([50], True)
        return sorted(np.nonzero(m.memory["sequence_priority"] != before)[0].tolist())

    assert changed(True) == [40, 50]       # reference: next neighbour typo idx - i
    assert changed(False) == [40, 50, 60]


def test_indexing_sample_contiguous_one_step_batches():
    """replay_memory.py:264-277 (unused by the reference, kept for API parity): 1-step batches
    over [start, last) with next_state n rows ahead, ring-wrapped."""
    m = _mem(10)
    for k in range(10):
        x = np.full((4, 84, 84), k * 20, dtype=np.uint8)
        m.add(x.astype(np.float32) / 255.0, np.zeros(256), np.zeros(256), np.zeros(256),
              np.zeros(256), k % 6, float(k), k == 9, 1, 0.1)
    batch, index = m.indexing_sample(6, 9)
    assert index.tolist() == [6, 7, 8]
    assert batch["state"].shape == (3, 1, 4, 84, 84)
    assert batch["state"][0, 0, 0, 0, 0] == pytest.approx(120 / 255)
    nxt = (index + m.n_step) % 10
    assert np.allclose(batch["next_state"][:, 0, 0, 0, 0], nxt * 20 / 255)
    assert batch["reward"][:, 0].tolist() == [6.0, 7.0, 8.0]


def test_extend_fit_and_wrap():
    m = _mem(10)
    src = {k: v[:7].copy() for k, v in _mem(7).memory.items()}
    src["reward"][:, 0] = np.arange(7)
    m.extend(src)
    m.extend(src)
    assert m.index == 14 and m.size == 10
    assert m.memory["reward"][:4, 0].tolist() == [3, 4, 5, 6]   # wrapped write
    m.fit()
    assert m.memory["state"].shape[0] == 10


def test_sample_contract_and_proportionality():
    rng = np.random.default_rng(0)
    m = _mem(400, burn_in=5, learning=5, seed=1)
    m.index = 400
    m.memory["priority"][:] = rng.random(400)
    starts = np.arange(0, 380, 10)
    m.memory["is_seq_start"][starts] = 1
    m.memory["sequence_priority"][starts] = 0.01
    m.memory["sequence_priority"][100] = 10.0   # one dominant sequence
    batch, seq, idx = m.sample()
    assert batch["state"].shape == (10, 4, 4, 84, 84) and batch["next_state"].shape == (10, 4, 4, 84, 84)
    assert batch["hs"].shape == (4, 256) and batch["target_cs"].shape == (4, 256)
    assert batch["action"].shape == (5, 4, 1) and batch["action"].dtype == torch.int64
    assert idx.shape == (10, 4) and np.all(idx[0] == seq)
    counts = sum((m.sample()[1] == 100).sum() for _ in range(200))
    assert counts / 800 > 0.9


def test_get_stacked_state_degenerate_and_padded():
    m = ReplayMemory(10, 2, 3, action_repeat=1, n_stacks=3, state_size=(2, 2))
    for i in range(6):
        m.add(np.full((1, 2, 2), i / 255.0), np.zeros(256), np.zeros(256), np.zeros(256),
              np.zeros(256), 0, 0, False, 3 if i == 0 else 1, 0)
    s = m.get_stacked_state(3)
    assert s.shape == (3, 2, 2) and [int(v) for v in s[:, 0, 0]] == [1, 2, 3]
    s0 = m._stacked(np.array([3]))[0]
    assert np.array_equal(s, s0)


def test_file_transport_roundtrip(tmp_path):
    a = _mem(50)
    for i in range(12):
        a.add(np.full((4, 84, 84), i / 255.0), np.full(256, i), np.zeros(256), np.zeros(256),
              np.zeros(256), i % 6, float(i), i == 11, 1, 0.1 * i)
    a.memory["is_seq_start"][[0, 2]] = 1
    assert a.save(str(tmp_path), 3)
    # a second save before the learner consumes appends (actor backlog merge)
    b = _mem(50)
    b.add(np.zeros((4, 84, 84)), np.zeros(256), np.zeros(256), np.zeros(256), np.zeros(256), 0, 99.0,
          False, 1, 1.0)
    assert b.save(str(tmp_path), 3)
    # tensor-only file: loadable with weights_only=True (Q2)
    d = torch.load(os.path.join(tmp_path, "memory3.pt"), weights_only=True)
    assert d["state"].shape[0] == 13
    learner = _mem(100)
    assert learner.load(str(tmp_path), 3) == 13
    assert not os.path.exists(os.path.join(tmp_path, "memory3.pt"))
    assert learner.memory["reward"][12, 0] == 99.0 and learner.memory["is_seq_start"][2] == 1
    assert learner.load(str(tmp_path), 3) == 0
