"""End-to-end bf16 HIP learner step vs the fp32 PyTorch autograd oracle (learner_ref.py)."""
import copy

import pytest
import torch

from pytorch_r2d2_amd.config import get_config
from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
from pytorch_r2d2_amd.learner_ref import batch_from_hbm, r2d2_loss
from pytorch_r2d2_amd.models import QNet

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _make(mode, B=16, preset="atari57", **kw):
    # the bf16 engine (the fp32 / split-precision engine: tests/test_split_gpu.py)
    over = {"learner.batch_size": B, "learner.target_mode": mode, "replay.capacity": 40000,
            "replay.n_subrings": 8, "learner.use_graph": False, "learner.compute_dtype": "bf16"}
    if preset == "atari57":
        over.update({"replay.burn_in": 6, "replay.learn": 8, "replay.overlap": 7})
    over.update(kw)
    cfg = get_config(preset, **over)
    rp = HBMReplay(cfg, DEV)
    rp.fill_synthetic(episode_len=100, seed=5)
    torch.manual_seed(7)
    net = QNet("cpu", cfg.model, cfg.env)
    tgt = QNet("cpu", cfg.model, cfg.env)  # different target weights exercise the target path
    eng = LearnerEngine(cfg, rp, DEV, init_module=net)
    eng.layout.load_state_dict(eng.target, tgt.state_dict())
    eng._pack(always=True)
    return cfg, rp, eng, net, tgt


@pytest.mark.parametrize("mode", ["shifted", "fixed", "reference"])
def test_engine_loss_and_grads_match_reference(mode):
    cfg, rp, eng, net, tgt = _make(mode)
    eng._forward_loss()
    eng._backward_core()
    eng._backward_torso()
    torch.cuda.synchronize()
    online = copy.deepcopy(net).to(DEV)
    target = copy.deepcopy(tgt).to(DEV)
    batch = batch_from_hbm(rp, eng.starts, eng.probs, cfg, DEV)
    out = r2d2_loss(online, target, batch, cfg, mode)
    out["loss"].backward()
    assert abs(eng.loss.item() - out["loss"].item()) / out["loss"].item() < 3e-2
    got = eng.layout.views(eng.grad)
    for name, p in online.named_parameters():
        r = _rel(got[name], p.grad)
        assert r < 8e-2, f"{name}: rel err {r}"
    # row priorities written back into the replay for the learning rows
    Lb, T = cfg.replay.burn_in, cfg.replay.seq_len
    s = eng.starts.long()
    base = s - s % rp.cap_e
    rows = base[None] + (s[None] - base[None] + torch.arange(Lb, T, device=DEV)[:, None]) % rp.cap_e
    assert _rel(rp.priority[rows], out["priority"]) < 5e-2


def test_engine_dmlab_rgb_torso_matches_reference():
    """DMLab-30 preset (3x72x96 RGB): the fused forward kernel instance for this geometry, then
    BOTH conv backwards from the same forward -- the fused torso_bwd.hip instance and the library
    (MIOpen) convolution_backward -- vs the fp32 autograd oracle.  bf16 operands put the conv1
    weight gradient near the 8 % bound for either backward, so the fused one must also stay within
    1.25x of the library's own error."""
    cfg, rp, eng, net, tgt = _make("shifted", B=8, preset="dmlab30",
                                   **{"replay.burn_in": 4, "replay.learn": 8, "replay.overlap": 6})
    assert not eng.fused_torso and eng.fwd_geom == (3, 72, 96)
    eng._forward_loss()
    eng._backward_core()
    core = eng.grad.clone()
    eng._backward_torso_fused()
    torch.cuda.synchronize()
    g_fused = eng.grad.clone()
    eng.grad.copy_(core)
    eng._backward_torso_library()
    torch.cuda.synchronize()
    g_lib = eng.grad.clone()
    online = copy.deepcopy(net).to(DEV)
    target = copy.deepcopy(tgt).to(DEV)
    batch = batch_from_hbm(rp, eng.starts, eng.probs, cfg, DEV)
    out = r2d2_loss(online, target, batch, cfg, "shifted")
    out["loss"].backward()
    assert abs(eng.loss.item() - out["loss"].item()) / out["loss"].item() < 3e-2
    got_f, got_l = eng.layout.views(g_fused), eng.layout.views(g_lib)
    for name, p in online.named_parameters():
        el, ef = _rel(got_l[name], p.grad), _rel(got_f[name], p.grad)
        assert el < 8e-2, (name, el)
        assert ef < max(8e-2, 1.25 * el), (name, ef, el)


def test_engine_graph_replay_matches_eager():
    cfg, rp, eng, net, tgt = _make("shifted", B=8)
    cfg2, rp2, eng2, _, _ = _make("shifted", B=8)
    for _ in range(3):
        eng.step_eager()
    eng2.capture(warmup=0)
    for _ in range(2):
        eng2.step()
    eng2.step_eager()  # capture() itself runs no step when warmup=0
    torch.cuda.synchronize()
    assert torch.equal(rp.step, rp2.step)
    assert _rel(eng2.master, eng.master) < 1e-5
    assert _rel(rp2.tree, rp.tree) < 1e-5


def test_engine_resume_from_full_checkpoint(tmp_path):
    from pytorch_r2d2_amd.utils.checkpoint import load_full_checkpoint, save_full_checkpoint
    cfg, rp, eng, net, tgt = _make("shifted", B=8)
    cfg2, rp2, eng2, _, _ = _make("shifted", B=8)
    for _ in range(3):
        eng.step_eager()
    path = str(tmp_path / "full.pt")
    save_full_checkpoint(path, eng.state_dict(), eng.target_state_dict(), None, 3, cfg,
                         eng.full_state_extra())
    for k, v in vars(rp).items():          # the replay is not part of the checkpoint
        if torch.is_tensor(v):
            getattr(rp2, k).copy_(v)
    for _ in range(2):
        eng.step_eager()
    eng2.load_full_state(load_full_checkpoint(path))
    for _ in range(2):
        eng2.step_eager()
    torch.cuda.synchronize()
    assert eng2.steps_done == 5
    assert _rel(eng2.master, eng.master) < 1e-6
    assert _rel(eng2.opt_a, eng.opt_a) < 1e-6


def test_engine_training_reduces_loss_on_fixed_batch():
    cfg, rp, eng, net, tgt = _make("shifted", B=16, **{"learner.lr": 3e-4})
    eng.step_eager()
    first = eng.loss.item()
    # freeze sampling to a fixed batch: shrink the tree to the first 16 sequences
    rp.tree[: rp.capacity] *= 0
    st = torch.nonzero(rp.is_start).squeeze(1)[:16]
    rp.tree[st] = 1.0
    rp.rebuild_tree()
    losses = []
    for _ in range(60):
        eng.step_eager()
        losses.append(eng.loss.item())
    assert min(losses[-10:]) < losses[0]


@pytest.mark.parametrize("preset", ["atari57", "dmlab30"])
def test_fused_torso_backward_matches_library(preset):
    """The fused torso backward (torso_bwd.hip, Atari 4x84x84 and DMLab-30 3x72x96 instances) vs
    MIOpen's convolution_backward from the same saved activations."""
    if preset == "atari57":
        cfg, rp, eng, net, tgt = _make("shifted", B=16)
    else:
        cfg, rp, eng, net, tgt = _make("shifted", B=8, preset="dmlab30",
                                       **{"replay.burn_in": 4, "replay.learn": 8, "replay.overlap": 6})
    eng._forward_loss()
    eng._backward_core()
    eng.grad.zero_()
    eng._backward_torso_library()
    torch.cuda.synchronize()
    ref = eng.grad.clone()
    eng.grad.zero_()
    eng._backward_torso_fused()
    torch.cuda.synchronize()
    L = eng.layout
    for name in ("vis_layers.0.weight", "vis_layers.0.bias", "vis_layers.2.weight",
                 "vis_layers.2.bias", "vis_layers.4.weight", "vis_layers.4.bias"):
        r = _rel(L.view(eng.grad, name), L.view(ref, name))
        assert r < 3e-2, f"{name}: rel err {r}"


@pytest.mark.parametrize("mode", ["shifted", "reference"])
def test_td_fused_head_backward_matches_separate_launches(mode):
    """td.hip td_duel_kernel (TD + dueling-head backward, a wave per transition) == td_kernel +
    head.hip dueling_bwd_kernel: dq, dz, dva, priorities and every gradient bit for bit, the loss
    to fp32 rounding (its partial sums are grouped differently)."""
    runs = []
    for fuse in (True, False):
        cfg, rp, eng, _, _ = _make(mode, B=64, **{"learner.td_fuse_head_bwd": fuse})
        eng._forward_loss()
        assert eng._duel_done == fuse
        eng._backward_core()
        eng._backward_torso()
        torch.cuda.synchronize()
        runs.append((eng, rp))
    (a, ra), (b, rb) = runs
    for name in ("dq", "dz", "dva", "td_abs", "is_w", "grad"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert torch.equal(ra.priority, rb.priority)
    assert abs(a.loss_value() - b.loss_value()) <= 1e-6 * max(1.0, abs(b.loss_value()))


def test_engine_bf16_seaquest_18_actions_fused_path():
    """bf16 engine, 18-action head (seaquest8 preset): TD + head backward fused (td_duel_kernel)
    and the head-gradient reduction in one gradsum launch -- no torch.mm fallback -- vs the fp32
    autograd oracle."""
    cfg, rp, eng, net, tgt = _make("fixed", preset="seaquest8",
                                   **{"replay.burn_in": 6, "replay.learn": 8, "replay.overlap": 7})
    assert eng.layout.A == 18
    calls = []
    orig = torch.mm
    torch.mm = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]   # noqa: E731
    try:
        eng._forward_loss()
        eng._backward_core()
        eng._backward_torso()
    finally:
        torch.mm = orig
    torch.cuda.synchronize()
    assert eng._duel_done
    assert not calls, len(calls)
    online = copy.deepcopy(net).to(DEV)
    target = copy.deepcopy(tgt).to(DEV)
    batch = batch_from_hbm(rp, eng.starts, eng.probs, cfg, DEV)
    out = r2d2_loss(online, target, batch, cfg, "fixed")
    out["loss"].backward()
    assert abs(eng.loss.item() - out["loss"].item()) / out["loss"].item() < 3e-2
    got = eng.layout.views(eng.grad)
    for name, p in online.named_parameters():
        r = _rel(got[name], p.grad)
        assert r < 8e-2, f"{name}: rel err {r}"


def test_td_fused_dh_matches_gemm():
    """td.hip r2_td_duel_dh: dh = dz @ W1 on the TD launch's MFMAs (16 rows per workgroup, W1^T
    from the packed head1T layout) vs the same product from the engine's dz in float64."""
    cfg, rp, eng, net, tgt = _make("shifted", B=16)
    eng._forward_loss()
    torch.cuda.synchronize()
    assert eng._dh_done
    N = eng.Ll * eng.B
    ref = eng.dz[:N].double() @ eng.pk["head1"].double()
    assert _rel(eng.dh[:N], ref) < 1e-5
