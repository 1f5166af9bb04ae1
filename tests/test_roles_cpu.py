"""Actor / learner roles (reference API), checkpointing, metrics, supervisor + fault injection."""
import os
import time

import numpy as np
import pytest
import torch

from pytorch_r2d2_amd.actor import Actor
from pytorch_r2d2_amd.config import get_config
from pytorch_r2d2_amd.learner import Learner
from pytorch_r2d2_amd.models import QNet
from pytorch_r2d2_amd.utils.checkpoint import (load_full_checkpoint, load_reference_checkpoint,
                                               save_full_checkpoint)


class ScriptEnv:
    """Deterministic env: reward = step index, episode of fixed length; obs (4,84,84)."""

    def __init__(self, length=12):
        self.length, self.t = length, 0

    def reset(self):
        self.t = 0
        return np.full((4, 84, 84), 0.5, dtype=np.float32)

    def step(self, a):
        self.t += 1
        return np.full((4, 84, 84), self.t / 255.0, dtype=np.float32), float(self.t), self.t >= self.length, {}


def _cfg(**kw):
    base = {"replay.burn_in": 2, "replay.learn": 3, "replay.overlap": 2, "learner.batch_size": 2,
            "learner.initial_exploration": 10}
    base.update(kw)
    return get_config("reference", **base)


def test_actor_emits_every_transition_with_nstep_returns(tmp_path):
    cfg = _cfg()
    a = Actor(0, 1, {}, "cpu", cfg=cfg, env=ScriptEnv(12), memory_path=str(tmp_path))
    for _ in range(12):
        a.step()
    m = a.replay_memory
    # all 12 transitions of the episode are stored (Q3 fixed), rewards are 3-step returns
    g = cfg.learner.gamma
    r = np.arange(1, 13, dtype=np.float64)
    exp = [sum(g ** i * r[k + i] for i in range(3) if k + i < 12) for k in range(12)]
    assert m.index == 12
    assert np.allclose(m.memory["reward"][:12, 0], exp, rtol=1e-5)
    assert m.memory["done"][:12, 0].tolist() == [0.0] * 9 + [1.0] * 3
    # sequence starts: range(0, 12-5, 2) + [7]
    assert np.nonzero(m.memory["is_seq_start"])[0].tolist() == [0, 2, 4, 6, 7]
    assert np.all(m.memory["sequence_priority"][[0, 2, 4, 6, 7]] > 0)


def test_actor_legacy_mode_reproduces_reference_loss_of_first_transition(tmp_path):
    cfg = _cfg()
    a = Actor(0, 1, {}, "cpu", cfg=cfg, env=ScriptEnv(12), memory_path=str(tmp_path), legacy=True)
    for _ in range(12):
        a.step()
    m = a.replay_memory
    assert m.index == 11                                  # first transition lost (Q3)
    tail = m.memory["reward"][8:11, 0]
    assert np.allclose(tail, tail[0])                     # identical tail returns (Q4)


def test_actor_pre_vs_post_stored_state(tmp_path):
    cfg = _cfg(**{"replay.stored_state": "pre"})
    a = Actor(0, 1, {}, "cpu", cfg=cfg, env=ScriptEnv(6), memory_path=str(tmp_path))
    a.step()
    a.step()
    a.step()
    a.step()
    m = a.replay_memory
    assert np.all(m.memory["hs_cs"][0] == 0)          # pre-step state of the first step is zero
    cfg2 = _cfg()
    b = Actor(0, 1, {}, "cpu", cfg=cfg2, env=ScriptEnv(6), memory_path=str(tmp_path))
    for _ in range(4):
        b.step()
    assert np.any(b.replay_memory.memory["hs_cs"][0] != 0)   # reference: post-step state (Q6)


def test_learner_torch_backend_trains_and_publishes(tmp_path):
    cfg = _cfg(**{"learner.save_dir": str(tmp_path / "save"), "learner.checkpoint_interval": 3,
                  "learner.publish_interval": 2})
    shared = {}
    L = Learner(1, shared, device="cpu", cfg=cfg, memory_path=str(tmp_path / "mem"),
                replay_capacity=500)
    assert shared["version"] == 1 and set(shared) >= {"net_state", "target_net_state"}
    a = Actor(0, 1, shared, "cpu", cfg=cfg, env=ScriptEnv(12), memory_path=str(tmp_path / "mem"))
    a.memory_save_interval = 2
    for _ in range(48):
        a.step()
    assert L.ingest() > 0
    w0 = {k: v.clone() for k, v in L.net.state_dict().items()}
    L.run(max_steps=4)
    assert L.n_epochs == 4
    assert any(not torch.equal(w0[k], v) for k, v in L.net.state_dict().items())
    assert shared["version"] >= 2
    # reference checkpoint at step 3 (save/ created: Q11), loads into a reference-shaped QNet
    sd = load_reference_checkpoint(str(tmp_path / "save" / "3_save.pt"))
    q = QNet()
    q.load_state_dict(sd)
    assert a.load_model()


def test_learner_resume_continues_identically(tmp_path):
    """Full-state checkpoint -> resume reproduces the uninterrupted run bit for bit (weights,
    target, centered-RMSprop moments, step counter and RNG streams restored; replay refilled)."""
    import copy
    cfg = _cfg(**{"learner.save_dir": str(tmp_path / "save"), "learner.checkpoint_interval": 10 ** 6})
    L1 = Learner(1, {}, device="cpu", cfg=cfg, memory_path=str(tmp_path / "mem"), replay_capacity=500)
    a = Actor(0, 1, {}, "cpu", cfg=cfg, env=ScriptEnv(12), memory_path=str(tmp_path / "mem"))
    a.memory_save_interval = 2
    for _ in range(60):
        a.step()
    assert L1.ingest() > 0
    L1.run(max_steps=3)
    ck = str(tmp_path / "full.pt")
    L1.save_checkpoint(ck)
    mem = copy.deepcopy(L1.replay_memory)
    L1.run(max_steps=5)            # run() takes an absolute step target
    L2 = Learner(1, {}, device="cpu", cfg=cfg, memory_path=str(tmp_path / "mem2"), replay_capacity=500)
    L2.replay_memory = mem
    assert L2.resume(ck) == 3
    L2.run(max_steps=5)
    assert L2.n_epochs == L1.n_epochs == 5
    for (k, v1), v2 in zip(L1.net.state_dict().items(), L2.net.state_dict().values()):
        assert torch.equal(v1, v2), k
    for g1, g2 in zip(L1.optim.state_dict()["state"].values(), L2.optim.state_dict()["state"].values()):
        assert torch.equal(g1["square_avg"], g2["square_avg"])


def test_full_checkpoint_roundtrip(tmp_path):
    q = QNet()
    opt = torch.optim.RMSprop(q.parameters(), lr=1e-3, centered=True)
    q(torch.rand(2, 4, 84, 84)).sum().backward()
    opt.step()
    p = save_full_checkpoint(str(tmp_path / "full.pt"), q.state_dict(), q.state_dict(), opt.state_dict(),
                             42, get_config("reference"))
    obj = load_full_checkpoint(p)
    assert obj["step"] == 42
    q2 = QNet()
    q2.load_state_dict(obj["online"])
    opt2 = torch.optim.RMSprop(q2.parameters(), lr=1e-3, centered=True)
    opt2.load_state_dict(obj["optimizer"])
    for a, b in zip(q.parameters(), q2.parameters()):
        assert torch.equal(a, b)


def test_inproc_cartpole_runs():
    from pytorch_r2d2_amd.runner import run_inproc
    cfg = get_config("cartpole", **{"learner.initial_exploration": 300, "learner.batch_size": 4,
                                    "replay.burn_in": 4, "replay.learn": 6, "replay.overlap": 5})
    out = run_inproc(cfg, steps=20, log_every=10)
    assert len(out["losses"]) == 2 and all(np.isfinite(out["losses"]))
    assert len(out["returns"]) > 0


def test_inproc_cartpole_learns():
    """BASELINE config 1 (CartPole-v1, seq 80 = burn-in 40 + learn 40, n=5, value rescaling, IS
    weights, stored state, on the CPU): 4 in-process actors + the fp32 torch learner.  A random
    policy balances ~20 steps; after 1800 learner steps the mean return of the last 20 episodes
    must be >= 150 (seeds 0 / 1 measured 206 at 1500 / 275 at 1800 steps, ~70 s on 8 CPUs)."""
    import random
    from pytorch_r2d2_amd.runner import run_inproc
    # every RNG and the intra-op thread count pinned: the outcome must not depend on which tests
    # ran before in the same process
    torch.manual_seed(0)
    np.random.seed(0)
    random.seed(0)
    nt = torch.get_num_threads()
    torch.set_num_threads(4)
    try:
        cfg = get_config("cartpole")
        out = run_inproc(cfg, steps=1800, n_actors=4, actor_steps_per_update=4, log_every=300)
    finally:
        torch.set_num_threads(nt)
    rets = out["returns"]
    # deterministic run: the learner's replay sampler is seeded from the config (it drew OS
    # entropy before, and this test passed or failed by chance); the same mean every run
    print(f"cartpole last-20 mean return {np.mean(rets[-20:]):.2f} over {len(rets)} episodes")
    assert len(rets) >= 40 and all(np.isfinite(out["losses"]))
    assert np.mean(rets[-20:]) >= 150, (np.mean(rets[:20]), np.mean(rets[-20:]))


def test_metrics_jsonl(tmp_path):
    from pytorch_r2d2_amd.utils.metrics import MetricsLogger, read_jsonl
    m = MetricsLogger(str(tmp_path / "m.jsonl"), rank=1)
    m.log("learner", step=1, loss=torch.tensor(0.5))
    m.close()
    rec = read_jsonl(str(tmp_path / "m.jsonl"))
    assert rec[0]["kind"] == "learner" and rec[0]["loss"] == 0.5 and rec[0]["rank"] == 1


def _crashy(i, beat=None):
    from pytorch_r2d2_amd.utils.faults import faults
    for step in range(1000):
        if beat:
            beat(step)
        faults().check("actor", i, step)
        time.sleep(0.005)


def _learner_like(seconds, beat=None):
    t0 = time.time()
    while time.time() - t0 < seconds:
        if beat:
            beat(0)
        time.sleep(0.01)


def _hangs(i, beat=None):
    from pytorch_r2d2_amd.utils.faults import faults
    for step in range(100000):
        if beat:
            beat(step)
        faults().check("actor", i, step)
        time.sleep(0.005)


def test_supervisor_restarts_crashed_actor_and_kills_stalled(monkeypatch):
    from pytorch_r2d2_amd.utils.supervisor import RoleSpec, Supervisor
    monkeypatch.setenv("R2D2_FAULTS", "actor:0:crash_at=20;actor:1:hang_at=20")
    roles = [RoleSpec("learner", _learner_like, (60.0,), restartable=False),
             RoleSpec("actor0", _crashy, (0,), max_restarts=2),
             RoleSpec("actor1", _hangs, (1,), max_restarts=8, stall_timeout_s=1.5)]
    sup = Supervisor(roles, poll_s=0.05)

    def done():
        # finished once actor0 used up its restarts (3 exits seen) and actor1 was caught stalling;
        # spawn start-up (a torch import per child) makes wall-clock budgets unreliable
        r = sup.report
        return len(r["actor0"]["exitcodes"]) >= 3 and r["actor1"]["stalls"] >= 1

    rep = sup.run(until=done, timeout_s=50)
    assert rep["actor0"]["restarts"] == 2
    assert 17 in rep["actor0"]["exitcodes"]
    assert rep["actor1"]["stalls"] >= 1


def test_once_fault_fires_in_first_incarnation_only(monkeypatch):
    """``once=1``: the restarted actor (R2D2_INCARNATION=1) runs past the crash step to a clean
    exit; the supervisor reports one restart and the exit codes [17, 0]."""
    from pytorch_r2d2_amd.utils.supervisor import RoleSpec, Supervisor
    monkeypatch.setenv("R2D2_FAULTS", "actor:0:crash_at=20,once=1")
    sup = Supervisor([RoleSpec("actor0", _crashy, (0,), max_restarts=3)], poll_s=0.05)
    rep = sup.run(timeout_s=60)
    assert rep["actor0"]["restarts"] == 1 and rep["actor0"]["exitcodes"] == [17, 0], rep
