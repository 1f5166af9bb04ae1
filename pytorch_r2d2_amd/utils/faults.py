"""Fault injection hooks (absent in the reference).

Faults are declared with the ``R2D2_FAULTS`` environment variable (inherited by spawned
processes) or programmatically, as ``;``-separated specs:

    actor:<id>:crash_at=<step>        hard-exit (os._exit(17)) when that actor reaches step
    actor:<id>:hang_at=<step>         stop beating (sleep forever) -> exercises the watchdog
    learner:0:crash_at=<step>
    push:<id>:drop=<prob>             drop a trajectory push with probability p
    weights:<id>:stale=<n>            ignore the first n weight publications
    dpcheck:<rank>:corrupt_at=<step>  perturb that rank's weight checksum in the one-graph DP
                                      rollout's validation at that step (parallel/graph_rollout.py)

Add ``once=1`` to a crash / hang rule (``actor:3:crash_at=500,once=1``) to fire it only in the
process's first incarnation: the supervisor exports ``R2D2_INCARNATION`` (its restart count) to
every child, so the restarted actor runs on instead of failing at the same step again.

Roles call ``faults().check(role, id, step)`` / ``faults().drop(role, id)``; with no spec the
calls are a dict lookup.
"""
from __future__ import annotations

import os
import random
import time
from typing import Dict, Tuple

EXIT_CODE = 17


class FaultPlan:
    def __init__(self, spec: str = ""):
        self.rules: Dict[Tuple[str, int], Dict[str, float]] = {}
        self.rng = random.Random(1234)
        for part in filter(None, (p.strip() for p in spec.split(";"))):
            role, rid, kv = part.split(":", 2)
            d = self.rules.setdefault((role, int(rid)), {})
            for item in kv.split(","):
                k, v = item.split("=")
                d[k] = float(v)

    def _r(self, role, rid):
        return self.rules.get((role, int(rid)))

    def check(self, role: str, rid: int, step: int) -> None:
        r = self._r(role, rid)
        if not r:
            return
        if r.get("once") and int(os.environ.get("R2D2_INCARNATION", "0")) > 0:
            return
        if "crash_at" in r and step >= r["crash_at"]:
            os._exit(EXIT_CODE)
        if "hang_at" in r and step >= r["hang_at"]:
            while True:
                time.sleep(3600)

    def drop(self, role: str, rid: int) -> bool:
        r = self._r(role, rid)
        return bool(r and "drop" in r and self.rng.random() < r["drop"])

    def corrupt(self, role: str, rid: int, step: int) -> bool:
        r = self._r(role, rid)
        return bool(r and "corrupt_at" in r and int(step) == int(r["corrupt_at"]))

    def stale(self, role: str, rid: int, n_seen: int) -> bool:
        r = self._r(role, rid)
        return bool(r and "stale" in r and n_seen < r["stale"])


_plan = None


def faults() -> FaultPlan:
    global _plan
    if _plan is None:
        _plan = FaultPlan(os.environ.get("R2D2_FAULTS", ""))
    return _plan


def set_faults(spec: str) -> FaultPlan:
    global _plan
    os.environ["R2D2_FAULTS"] = spec
    _plan = FaultPlan(spec)
    return _plan


class Liveness:
    """Per-role liveness hook: fault-injection check every tick, heartbeat (supervisor
    ``Beat``) at most every ``every_s`` seconds.  Roles call ``tick(step)`` once per iteration."""

    def __init__(self, role: str, rid: int, beat=None, every_s: float = 0.25):
        self.role, self.rid, self.beat, self.every_s = role, int(rid), beat, every_s
        self._last = 0.0

    def tick(self, step: int, status: int = 0) -> None:
        faults().check(self.role, self.rid, step)
        if self.beat is not None:
            now = time.monotonic()
            if now - self._last >= self.every_s:
                self._last = now
                self.beat(int(step), status)
