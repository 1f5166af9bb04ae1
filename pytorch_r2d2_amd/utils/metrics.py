"""Structured metrics (JSONL) -- SURVEY §5.5.  The reference only prints (actor.py:110,
learner.py:59).  Every record is one JSON object per line: {"ts", "kind", "rank", ...fields}."""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Any, Dict, Optional


class MetricsLogger:
    def __init__(self, path: Optional[str], rank: int = 0, flush_every: int = 1):
        self.path = path
        self.rank = rank
        self._f = None
        self._n = 0
        self._flush_every = flush_every
        self._lock = threading.Lock()
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self._f = open(path, "a", buffering=1)

    def log(self, kind: str, **fields: Any) -> Dict[str, Any]:
        rec = {"ts": time.time(), "kind": kind, "rank": self.rank}
        for k, v in fields.items():
            if hasattr(v, "item"):
                v = v.item()
            rec[k] = v
        if self._f is not None:
            with self._lock:
                self._f.write(json.dumps(rec) + "\n")
                self._n += 1
                if self._n % self._flush_every == 0:
                    self._f.flush()
        return rec

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None


def read_jsonl(path: str):
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]


class RateMeter:
    """Exponentially smoothed events/s."""

    def __init__(self, alpha: float = 0.1):
        self.alpha = alpha
        self.rate = 0.0
        self._t = None

    def update(self, n: float = 1.0) -> float:
        now = time.perf_counter()
        if self._t is not None:
            dt = max(now - self._t, 1e-9)
            r = n / dt
            self.rate = r if self.rate == 0 else (1 - self.alpha) * self.rate + self.alpha * r
        self._t = now
        return self.rate
