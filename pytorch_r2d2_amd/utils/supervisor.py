"""Process supervisor with failure detection and actor restarts.

The reference starts the learner and N actors and joins them forever (main.py:29-33): a
crashed actor is never noticed and the learner spins.  ``Supervisor``:

* starts every role as a ``spawn`` child with a heartbeat slot in a shared-memory
  ``HeartbeatTable`` (native runtime);
* polls exit codes and heartbeat ages; a dead or stalled *actor* is restarted (up to
  ``max_restarts`` each, with the same id so it resumes its epsilon and file slot); a dead or
  stalled *learner* stops the job (its state lives in checkpoints);
* ``run(until=...)`` returns a report {role: {restarts, exitcodes}}.

Children call ``heartbeat(slot, counter)`` through the ``Beat`` helper passed in their kwargs.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..runtime import HeartbeatTable


class Beat:
    """Picklable heartbeat handle given to children."""

    def __init__(self, table_name: str, n_slots: int, slot: int):
        self.table_name, self.n_slots, self.slot = table_name, n_slots, slot
        self._t = None

    def __call__(self, counter: int = 0, status: int = 0):
        if self._t is None:
            self._t = HeartbeatTable(self.table_name, self.n_slots, create=False)
        self._t.beat(self.slot, counter, status)


@dataclass
class RoleSpec:
    name: str
    target: Callable
    args: tuple = ()
    kwargs: Dict[str, Any] = field(default_factory=dict)
    restartable: bool = True
    stall_timeout_s: float = 0.0     # 0 = no heartbeat watchdog
    max_restarts: int = 3


def _child_entry(target, args, kwargs, beat: Beat, incarnation: int = 0):
    import inspect
    os.environ["R2D2_INCARNATION"] = str(incarnation)    # read by utils/faults.py once-rules
    beat(0, 1)
    kwargs = dict(kwargs)
    try:
        if "beat" in inspect.signature(target).parameters:
            kwargs.setdefault("beat", beat)
    except (TypeError, ValueError):
        pass
    target(*args, **kwargs)


class Supervisor:
    def __init__(self, roles: List[RoleSpec], poll_s: float = 0.2, start_method: str = "spawn"):
        self.roles = roles
        self.poll_s = poll_s
        self.ctx = mp.get_context(start_method)
        self.table_name = f"/r2d2_hb_{os.getpid()}_{uuid.uuid4().hex[:8]}"
        self.table = HeartbeatTable(self.table_name, max(1, len(roles)), create=True)
        self.procs: List[Optional[mp.Process]] = [None] * len(roles)
        self.report = {r.name: {"restarts": 0, "exitcodes": [], "stalls": 0} for r in roles}
        self.started_at = [0.0] * len(roles)

    def _start(self, i: int):
        r = self.roles[i]
        beat = Beat(self.table_name, len(self.roles), i)
        p = self.ctx.Process(target=_child_entry, args=(r.target, r.args, r.kwargs, beat,
                                                               self.report[r.name]["restarts"]),
                             name=r.name, daemon=False)
        p.start()
        self.procs[i] = p
        self.started_at[i] = time.monotonic()

    def start(self):
        for i in range(len(self.roles)):
            self._start(i)

    def _stalled(self, i: int) -> bool:
        r = self.roles[i]
        if r.stall_timeout_s <= 0:
            return False
        age = self.table.age_s(i)
        since_start = time.monotonic() - self.started_at[i]
        return since_start > r.stall_timeout_s and age > r.stall_timeout_s

    def poll(self) -> bool:
        """One supervision pass.  Returns False when the job must stop."""
        for i, (r, p) in enumerate(zip(self.roles, self.procs)):
            if p is None:
                continue
            dead = not p.is_alive()
            stalled = (not dead) and self._stalled(i)
            if not dead and not stalled:
                continue
            if stalled:
                self.report[r.name]["stalls"] += 1
                p.kill()
                p.join(5)
            else:
                p.join(0.1)
            self.report[r.name]["exitcodes"].append(p.exitcode)
            if p.exitcode == 0 and not stalled:
                self.procs[i] = None       # clean exit
                continue
            if r.restartable and self.report[r.name]["restarts"] < r.max_restarts:
                self.report[r.name]["restarts"] += 1
                self._start(i)
            else:
                return False
        return any(p is not None for p in self.procs)

    def run(self, until: Optional[Callable[[], bool]] = None, timeout_s: Optional[float] = None):
        self.start()
        t0 = time.monotonic()
        try:
            while True:
                ok = self.poll()
                if not ok:
                    break
                if until is not None and until():
                    break
                if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                    break
                time.sleep(self.poll_s)
        finally:
            self.stop()
        return self.report

    def stop(self):
        for p in self.procs:
            if p is not None and p.is_alive():
                p.terminate()
        for p in self.procs:
            if p is not None:
                p.join(10)
                if p.is_alive():
                    p.kill()
                    p.join(5)
        self.table.close(unlink=True)
