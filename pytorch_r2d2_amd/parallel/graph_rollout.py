"""When may the data-parallel learner step run as ONE captured graph (collectives included)?

The DP step has two captured forms (engine/learner_engine.py ``capture``):

    segments   4-6 graphs with the RCCL bucket all-reduces / the shard-stats all-gather issued
               between them on the communication stream -- the form the multi-rank tests pin;
    one graph  the collectives captured on their side streams (fork / join as graph edges): the
               segment boundaries' ~15 us each disappear (profiles/r03_force_dp_ab.txt: the DP
               machinery's overhead at one forced rank 1.180 -> 1.122 ms).

No multi-rank RCCL run has validated the one-graph form on this hardware, so it is rolled out per
run (round-6 verdict item 7; reference: a single learner, /root/reference/learner.py:19):

  1. the first ``warm`` steps replay the segment graphs;
  2. then the one graph is captured and replayed; for ``validate`` steps every rank records a
     checksum of its weights and its error word on the device (no host sync per step), and at the
     end of the window ONE all-reduce (MAX) of ``[checksums, -checksums, error words]`` decides:
     identical weights on every rank give max - min = 0 at every step;
  (a capture that raises on any rank -- agreed by one all-reduce -- keeps every rank on the
  segment graphs;)
  3. any mismatch or a non-zero error word switches EVERY rank back to the segment graphs for the
     rest of the run (the decision is taken on the all-reduced values, so all ranks agree), the
     engine re-broadcasts rank 0's weights / optimizer state, and ``fallback`` is reported
     (bench.py labels its JSON line with ``label()``).

At world 1 (the --force-dp rehearsal) there is nothing to compare: the one graph is used after
the warm-up steps without a validation window.

``R2D2_FAULTS="dpcheck:<rank>:corrupt_at=<step>"`` perturbs that rank's checksum at that step
(utils/faults.py) -- how the fallback path is exercised (tests/test_dist_cpu.py).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..utils.faults import faults


class GraphRollout:
    def __init__(self, group, rank: int, world: int, enabled: bool, warm: int = 3,
                 validate: int = 50, device=None):
        self.group, self.rank, self.world = group, int(rank), int(world)
        self.enabled = bool(enabled)
        self.warm = int(warm)
        self.validate = int(validate) if world > 1 else 0
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.mode = "segments"
        self.fallback = False
        self.checked = 0
        self.mismatch_step: Optional[int] = None
        self.refusal: Optional[str] = None
        self._buf = None
        self._steps = []

    def want_promote(self, steps_done: int) -> bool:
        """Capture and switch to the one graph now (after the warm-up segment steps)?"""
        return (self.enabled and not self.fallback and self.mode == "segments"
                and steps_done >= self.warm)

    def agree(self, ok: bool) -> bool:
        """Did the one-graph capture succeed on EVERY rank?  One all-reduce (MIN) of the local
        flag, issued outside any capture: a rank whose capture raised keeps every rank on the
        segment graphs (their collective sequences must stay identical)."""
        if not (dist.is_initialized() and self.world > 1):
            return bool(ok)
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(t.item()))

    def refused(self, reason: str) -> None:
        """The one graph could not be captured (on some rank): segments for the rest of the run."""
        self.mode = "segments"
        self.fallback = True
        self.refusal = reason

    def promoted(self) -> None:
        self.mode = "one"
        self.checked = 0
        self._steps = []
        if self.validate:
            # [checksums | -checksums | error words], one slot per validation step
            self._buf = torch.zeros(3 * self.validate, dtype=torch.float64, device=self.device)

    def validating(self) -> bool:
        return self.mode == "one" and self.checked < self.validate

    def record(self, checksum: torch.Tensor, err: torch.Tensor, step: int) -> Optional[bool]:
        """One validation step (every rank, same step): device-side writes only.  At the end of
        the window returns the verdict (True = all ranks agreed at every step), else None."""
        i, v = self.checked, self.validate
        c = checksum.detach().reshape(()).to(self._buf.device, torch.float64)
        if faults().corrupt("dpcheck", self.rank, step):
            c = c + 1.0
        self._buf[i] = c
        self._buf[v + i] = -c
        self._buf[2 * v + i] = err.detach().reshape(()).to(self._buf.device, torch.float64)
        self._steps.append(int(step))
        self.checked += 1
        if self.checked < v:
            return None
        return self.conclude()

    def conclude(self) -> bool:
        t = self._buf
        if dist.is_initialized() and self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        v = self.validate
        h = t.cpu()
        spread = h[:v] + h[v:2 * v]          # max - min of each step's checksum over the ranks
        bad = (spread != 0) | (h[2 * v:] != 0)
        if bool(bad.any()):
            self.mode = "segments"
            self.fallback = True
            self.mismatch_step = self._steps[int(torch.nonzero(bad)[0])]
            return False
        return True

    def label(self) -> str:
        if self.refusal is not None:
            return "segment graphs (one-graph capture refused: %s)" % self.refusal
        if self.fallback:
            return "segment graphs (one-graph fallback at step %d)" % self.mismatch_step
        if self.mode == "one":
            if self.validate and self.validating():
                return "one graph, RCCL captured (validating)"
            return ("one graph, RCCL captured (validated over %d steps)" % self.validate
                    if self.validate else "one graph, RCCL captured")
        return "segment graphs"
