"""Host (numpy) prioritized sequence replay with the reference API.

Parity target: ``ReplayMemory`` in ``/root/reference/replay_memory.py:58-277`` -- same
constructor arguments, the same ``memory`` dict schema (state uint8 (4,84,84),
hs_cs / target_hs_cs f32 (512,), action int8, reward f32, done f32, stack_count int8, priority,
sequence_priority, is_seq_start) and the same methods: ``add extend fit save load
update_priority set_hs_cs update_sequence_priority get_stacked_state sample indexing_sample
size index memory``.

This is the compatibility / CPU path (CPU actors, the CartPole plumbing config, reading the
reference's actor files).  On MI355X the learner uses ``engine.replay_hbm.HBMReplay`` (same
schema, resident in HBM, GPU sum tree).

Fixed by default (``legacy=True`` restores the reference behaviour for comparison tests):
  Q2 -- transport files are written atomically under a separate fcntl lock file and contain only
        tensors (loadable with ``torch.load(weights_only=True)``); a failed load is reported and
        the file is kept instead of being silently deleted.
  Q8 -- the "next neighbour" refresh looks forward (idx + i), not backward (idx - i).
  Q9 -- sequence-priority windows wrap around the ring end.
  quantisation uses rint (state*255 round trip is exact even when x/255*255 < k in float32).
Sampling is vectorised (one cumsum + searchsorted instead of ``WeightedRandomSampler`` + 2*T*B
Python ``get_stacked_state`` calls, replay_memory.py:224-262).
"""
from __future__ import annotations

import os
import tempfile
from time import sleep
from typing import Dict, Optional

import numpy as np
import torch

from ..runtime import FileLock


class ReplayMemory:
    KEYS = ("state", "hs_cs", "target_hs_cs", "action", "reward", "done", "stack_count",
            "priority", "sequence_priority", "is_seq_start")

    def __init__(self, memory_size=100000, batch_size=32, n_step=3, state_size=(84, 84),
                 cell_size=256, action_repeat=4, n_stacks=4, alpha=0.4, *, burn_in=10,
                 learning=10, eta=0.9, legacy=False, obs_shape=None, obs_dtype=np.uint8,
                 seed=None):
        self.index = 0
        self.memory_size = memory_size
        self.cell_size = cell_size
        self.batch_size = batch_size
        self.n_step = n_step
        self.state_size = tuple(obs_shape) if obs_shape is not None else (action_repeat,) + tuple(state_size)
        self.obs_dtype = np.dtype(obs_dtype)
        self.action_repeat = action_repeat
        self.n_stacks = max(1, n_stacks // action_repeat)
        self.alpha = alpha
        self.beta = 0.4
        self.beta_step = 0.00025 / 4
        self.eta = eta
        self.burn_in_length = burn_in
        self.learning_length = learning
        self.sequence_length = burn_in + learning
        self.legacy = legacy
        self.rng = np.random.default_rng(seed)
        m = dict()
        m["state"] = np.zeros((memory_size, *self.state_size), dtype=self.obs_dtype)
        m["hs_cs"] = np.zeros((memory_size, cell_size * 2), dtype=np.float32)
        m["target_hs_cs"] = np.zeros((memory_size, cell_size * 2), dtype=np.float32)
        m["action"] = np.zeros((memory_size, 1), dtype=np.int8)
        m["reward"] = np.zeros((memory_size, 1), dtype=np.float32)
        m["done"] = np.zeros((memory_size, 1), dtype=np.float32)
        m["stack_count"] = np.zeros((memory_size,), dtype=np.int8)
        m["priority"] = np.zeros((memory_size,), dtype=np.float32)
        m["sequence_priority"] = np.zeros((memory_size,), dtype=np.float32)
        m["is_seq_start"] = np.zeros((memory_size,), dtype=np.uint8)
        self.memory = m
        self.arange = np.arange(memory_size)

    # ------------------------------------------------------------------ basic ring ops
    @property
    def size(self) -> int:
        return min(self.index, self.memory_size)

    def _quantize(self, state):
        if self.obs_dtype == np.uint8:
            return np.rint(np.asarray(state, dtype=np.float32) * 255.0).clip(0, 255).astype(np.uint8)
        return np.asarray(state, dtype=self.obs_dtype)

    def add(self, state, hs, cs, target_hs, target_cs, action, reward, done, stack_count, priority):
        """replay_memory.py:93-105."""
        i = self.index % self.memory_size
        m, c = self.memory, self.cell_size
        m["state"][i] = self._quantize(state)
        m["hs_cs"][i, :c] = np.asarray(hs).reshape(-1)
        m["hs_cs"][i, c:] = np.asarray(cs).reshape(-1)
        m["target_hs_cs"][i, :c] = np.asarray(target_hs).reshape(-1)
        m["target_hs_cs"][i, c:] = np.asarray(target_cs).reshape(-1)
        m["action"][i] = action
        m["reward"][i] = reward
        m["done"][i] = 1 if done else 0
        m["stack_count"][i] = stack_count
        m["priority"][i] = priority
        m["is_seq_start"][i] = 0          # a recycled row is no longer a sequence start
        m["sequence_priority"][i] = 0
        self.index += 1

    def extend(self, memory: Dict[str, np.ndarray]):
        """Bulk ring write of another memory dict (replay_memory.py:107-119)."""
        n = int(memory["state"].shape[0])
        if n == 0:
            return
        start = self.index % self.memory_size
        idx = (start + np.arange(n)) % self.memory_size
        if n > self.memory_size:  # only the newest rows survive
            idx = idx[-self.memory_size:]
            sl = slice(n - self.memory_size, n)
        else:
            sl = slice(0, n)
        for key in self.memory.keys():
            if key in memory:
                self.memory[key][idx] = np.asarray(memory[key])[sl]
        self.index += n

    def fit(self):
        for key in self.memory.keys():
            self.memory[key] = self.memory[key][: self.size]

    def update_priority(self, index, priority):
        self.memory["priority"][np.asarray(index)] = np.asarray(priority).reshape(-1)

    def set_hs_cs(self, index, hs, cs, target_hs, target_cs):
        c = self.cell_size
        self.memory["hs_cs"][index, :c] = hs
        self.memory["hs_cs"][index, c:] = cs
        self.memory["target_hs_cs"][index, :c] = target_hs
        self.memory["target_hs_cs"][index, c:] = target_cs

    # ------------------------------------------------------------------ sequence priorities
    def _mix(self, idx: int) -> float:
        cap = self.memory_size if not self.legacy else len(self.memory["priority"])
        if self.legacy:  # Q9: slice ignores ring wrap
            p = self.memory["priority"][idx: idx + self.sequence_length]
        else:
            p = self.memory["priority"][(idx + np.arange(self.sequence_length)) % cap]
        if p.size == 0:
            return 0.0
        return float(self.eta * p.max() + (1 - self.eta) * p.mean())

    def update_sequence_priority(self, index, update_pre_next_seq_priority=False):
        """replay_memory.py:184-213 (Q8/Q9 fixed unless legacy)."""
        cap = len(self.memory["priority"])
        starts = self.memory["is_seq_start"]
        for idx in np.asarray(index).reshape(-1):
            idx = int(idx)
            self.memory["sequence_priority"][idx % cap] = self._mix(idx % cap)
            if not update_pre_next_seq_priority:
                continue
            for i in range(1, self.sequence_length + 1):
                if starts[(idx - i) % cap] == 1:
                    pre = (idx - i) % cap
                    self.memory["sequence_priority"][pre] = self._mix(pre)
                    break
            for i in range(1, self.sequence_length + 1):
                if starts[(idx + i) % cap] == 1:
                    nxt = (idx - i) if self.legacy else (idx + i)  # Q8
                    nxt %= cap
                    self.memory["sequence_priority"][nxt] = self._mix(nxt)
                    break

    # ------------------------------------------------------------------ batch building
    def get_stacked_state(self, index):
        """replay_memory.py:215-222."""
        stack_count = int(self.memory["stack_count"][index])
        start = index - (self.n_stacks - stack_count)
        if start < 0:
            start = self.memory_size + start
        stack_index = [start for _ in range(stack_count)] + \
            [(start + 1 + i) % self.memory_size for i in range(self.n_stacks - stack_count)]
        return np.concatenate([self.memory["state"][i] for i in stack_index])

    def _stacked(self, rows: np.ndarray) -> np.ndarray:
        """Vectorised get_stacked_state over an index array of any shape."""
        if self.n_stacks == 1:
            return self.memory["state"][rows]
        sc = self.memory["stack_count"][rows].astype(np.int64)
        start = (rows - (self.n_stacks - sc)) % self.memory_size
        parts = []
        for k in range(self.n_stacks):
            r = np.where(k < sc, start, (start + 1 + (k - sc)) % self.memory_size)
            parts.append(self.memory["state"][r])
        return np.concatenate(parts, axis=-3)

    def sample_indices(self, batch_size: Optional[int] = None):
        starts = self.arange[: len(self.memory["is_seq_start"])][self.memory["is_seq_start"] == 1]
        if starts.size == 0:
            raise RuntimeError("no complete sequences in replay")
        p = self.memory["sequence_priority"][starts].astype(np.float64)
        if p.sum() <= 0:
            p = np.ones_like(p)
        c = np.cumsum(p)
        u = self.rng.random(batch_size or self.batch_size) * c[-1]
        pick = np.minimum(np.searchsorted(c, u, side="right"), starts.size - 1)
        return starts[pick], p[pick] / c[-1], starts.size

    def sample(self, device="cpu", return_probs: bool = False):
        """replay_memory.py:224-262: (batch, seq_index, index)."""
        seq_index, probs, n_valid = self.sample_indices()
        cap = self.memory_size
        T, Lb, Ll = self.sequence_length, self.burn_in_length, self.learning_length
        next_seq = (seq_index + self.n_step) % cap
        tt = np.arange(T)[:, None]
        rows = (seq_index[None, :] + tt) % cap                       # (T, B)
        nrows = (next_seq[None, :] + tt) % cap
        lrows = (seq_index[None, :] + Lb + np.arange(Ll)[:, None]) % cap
        m, c = self.memory, self.cell_size
        scale = 1.0 / 255.0 if self.obs_dtype == np.uint8 else 1.0
        batch = {
            "state": torch.from_numpy(self._stacked(rows).astype(np.float32) * scale),
            "next_state": torch.from_numpy(self._stacked(nrows).astype(np.float32) * scale),
            "hs": torch.from_numpy(m["hs_cs"][seq_index, :c]),
            "cs": torch.from_numpy(m["hs_cs"][seq_index, c:]),
            "target_hs": torch.from_numpy(m["target_hs_cs"][next_seq, :c]),
            "target_cs": torch.from_numpy(m["target_hs_cs"][next_seq, c:]),
            # extras (not in the reference batch): stored states for the other target modes
            "target_hs0": torch.from_numpy(m["target_hs_cs"][seq_index, :c]),
            "target_cs0": torch.from_numpy(m["target_hs_cs"][seq_index, c:]),
            "next_hs": torch.from_numpy(m["hs_cs"][next_seq, :c]),
            "next_cs": torch.from_numpy(m["hs_cs"][next_seq, c:]),
            "action": torch.from_numpy(m["action"][lrows].astype(np.int64)),
            "reward": torch.from_numpy(m["reward"][lrows].astype(np.float32)),
            "done": torch.from_numpy(m["done"][lrows].astype(np.float32)),
        }
        batch = {k: v.to(device) for k, v in batch.items()}
        if return_probs:
            return batch, seq_index, rows, probs, n_valid
        return batch, seq_index, rows

    def indexing_sample(self, start_index, last_index, device="cpu"):
        index = np.arange(start_index, last_index) % self.memory_size
        next_index = (index + self.n_step) % self.memory_size
        scale = 1.0 / 255.0 if self.obs_dtype == np.uint8 else 1.0
        batch = {
            "state": self._stacked(index)[:, None].astype(np.float32) * scale,
            "next_state": self._stacked(next_index)[:, None].astype(np.float32) * scale,
            "action": self.memory["action"][index],
            "reward": self.memory["reward"][index],
            "done": self.memory["done"][index],
        }
        return batch, index

    # ------------------------------------------------------------------ file transport
    @staticmethod
    def _to_tensors(mem: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
        return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in mem.items()}

    @staticmethod
    def read_file(path: str, allow_pickle: bool = False) -> Dict[str, np.ndarray]:
        """Load a transport file.  Our files hold only tensors (weights_only=True).  Files written
        by the reference (a pickled dict of numpy arrays) need ``allow_pickle=True`` -- only for
        files you trust."""
        try:
            d = torch.load(path, map_location="cpu", weights_only=True)
        except Exception:
            if not allow_pickle:
                raise
            d = torch.load(path, map_location="cpu", weights_only=False)  # opt-in, trusted only
        return {k: (v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)) for k, v in d.items()}

    def save(self, path, actor_id, blocking: bool = True, retry_sleep: float = 0.05):
        """Actor side of the file transport (replay_memory.py:125-152): merge with an unconsumed
        file under the lock, then write atomically (tmp + rename)."""
        os.makedirs(path, exist_ok=True)
        fpath = os.path.join(path, f"memory{actor_id}.pt")
        lock = FileLock(fpath)
        try:
            while not lock.acquire(blocking=False):
                if not blocking:
                    return False
                sleep(retry_sleep)
            if os.path.isfile(fpath) and os.path.getsize(fpath) > 0:
                old = self.read_file(fpath)
                mem = {k: np.concatenate([old[k], self.memory[k][: self.size]]) for k in self.memory}
            else:
                mem = {k: v[: self.size] for k, v in self.memory.items()}
            fd, tmp = tempfile.mkstemp(dir=path, suffix=".tmp")
            os.close(fd)
            torch.save(self._to_tensors(mem), tmp)
            os.replace(tmp, fpath)
            return True
        finally:
            lock.release()
            lock.close()

    def load(self, path, actor_id, allow_pickle: bool = False) -> int:
        """Learner side (replay_memory.py:155-173): ingest + delete under the lock; returns rows
        ingested (0 if no file or the lock is busy)."""
        fpath = os.path.join(path, f"memory{actor_id}.pt")
        if not (os.path.isfile(fpath) and os.path.getsize(fpath) > 0):
            return 0
        lock = FileLock(fpath)
        try:
            if not lock.acquire(blocking=False):
                return 0
            mem = self.read_file(fpath, allow_pickle=allow_pickle)
            self.extend(mem)
            os.remove(fpath)
            return int(mem["state"].shape[0])
        finally:
            lock.release()
            lock.close()
