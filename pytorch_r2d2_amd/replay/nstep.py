"""n-step transition builder.

Parity target: ``NStepMemory`` in ``/root/reference/replay_memory.py:12-55`` (API: ``add``,
``get``, ``size``, ``is_full``; parallel deques of q, state, hs, cs, target_hs, target_cs,
action, reward, stack_count).

Two behaviours:

* ``legacy=True`` reproduces the reference exactly, including
  Q3 -- every deque has ``maxlen=n`` so the 4th ``add`` evicts the first transition before it is
  ever emitted (the first transition of every episode is lost), and
  Q4 -- ``get`` never pops the reward deque and sums ALL buffered rewards, so the tail flush at
  episode end gives the last transitions identical returns.
* default (fixed): nothing is evicted implicitly; ``get`` pops the oldest transition and returns
  its discounted return over the (up to n) rewards that follow it, so the tail flush yields
  correctly truncated returns.
"""
from __future__ import annotations

from collections import deque


class NStepMemory(dict):
    FIELDS = ("q_value", "state", "hs", "cs", "target_hs", "target_cs", "action", "reward",
              "stack_count")

    def __init__(self, memory_size: int = 3, gamma: float = 0.99, legacy: bool = False):
        super().__init__()
        self.memory_size = memory_size
        self.gamma = gamma
        self.legacy = legacy
        maxlen = memory_size if legacy else None
        for f in self.FIELDS:
            setattr(self, f, deque(maxlen=maxlen))

    @property
    def size(self) -> int:
        return len(self.state)

    def add(self, q_value, state, hs, cs, target_hs, target_cs, action, reward, stack_count):
        for f, v in zip(self.FIELDS, (q_value, state, hs, cs, target_hs, target_cs, action, reward,
                                      stack_count)):
            getattr(self, f).append(v)

    def nstep_return(self) -> float:
        if self.legacy:
            return sum(self.gamma ** i * r for i, r in enumerate(self.reward))
        return sum(self.gamma ** i * r for i, r in enumerate(list(self.reward)[: self.memory_size]))

    def get(self):
        reward = self.nstep_return()
        out = []
        for f in self.FIELDS:
            if f == "reward":
                if not self.legacy:
                    self.reward.popleft()
                out.append(reward)
            else:
                out.append(getattr(self, f).popleft())
        # order of the reference tuple: q, state, hs, cs, target_hs, target_cs, action, reward,
        # stack_count (replay_memory.py:52)
        return tuple(out)

    def is_full(self) -> bool:
        return len(self.state) == self.memory_size
