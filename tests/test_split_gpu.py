"""Split precision (compute_dtype "fp32", csrc/split.h): fp32-accurate products on the bf16
matrix cores.  Kernels and the whole learner step are compared against float64 PyTorch
references; the bar is the fp32 one (rel <= 1e-4 end to end, ~1e-5 per GEMM)."""
import copy

import pytest
import torch

from pytorch_r2d2_amd.ops.gemm import Gemm, gemm, gemm_group, group_ws_bytes

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-300)).item()


def _split(x):
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return hi, lo


def _op(rows, cols, kmajor, gen):
    x = torch.randn(rows, cols, generator=gen, device=DEV)
    return x if kmajor else x.t().contiguous().t()


@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 0)])
@pytest.mark.parametrize("M,N,K", [(5440, 1024, 1568), (2560, 512, 256), (304, 200, 128), (2560, 256, 512)])
def test_split_gemm_is_fp32_accurate(ak, bk, M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M + N + K + ak)
    a = _op(M, K, ak, g)
    b = _op(N, K, bk, g).t()
    ah, al = _split(a)
    bh, bl = _split(b)
    c = torch.empty(M, N, device=DEV)
    bias = torch.randn(N, generator=g, device=DEV)
    gemm(Gemm(ah, bh, c, bias=bias, a_lo=al, b_lo=bl))
    ref = a.double() @ b.double() + bias.double()
    torch.cuda.synchronize()
    r = _rel(c, ref)
    assert r < 2e-5, r
    # bf16 operands alone are ~1e-3 off: the lo passes are what buys the accuracy
    c1 = torch.empty(M, N, device=DEV)
    gemm(Gemm(ah, bh, c1, bias=bias))
    assert _rel(c1, ref) > 20 * r


def test_split_gemm_split_output_and_group():
    """C written as hi / lo planes (the dX GEMM); the grouped weight-gradient launch with split
    operands, K split 1 and 2 ways."""
    g = torch.Generator(device=DEV).manual_seed(5)
    M, N, K = 2560, 1568, 1024
    a, b = _op(M, K, 1, g), _op(N, K, 0, g).t()
    ah, al = _split(a)
    bh, bl = _split(b)
    ch = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    cl = torch.empty_like(ch)
    gemm(Gemm(ah, bh, ch, a_lo=al, b_lo=bl, c_lo=cl))
    ref = a.double() @ b.double()
    torch.cuda.synchronize()
    assert _rel(ch.double() + cl.double(), ref) < 2e-5
    probs, refs = [], []
    for (M, N, K) in [(1024, 1568, 2560), (1024, 256, 2560), (512, 256, 2560)]:
        x = _op(K, M, 1, g).t()          # mn-major A (dgates^T)
        y = _op(N, K, 0, g).t()          # mn-major B (X)
        xh, xl = _split(x)
        yh, yl = _split(y)
        c = torch.zeros(M, N, device=DEV)
        probs.append(Gemm(xh, yh, c, a_lo=xl, b_lo=yl))
        refs.append(x.double() @ y.double())
    for splits in ([1, 1, 1], [2, 1, 2]):
        for p in probs:
            p.c.zero_()
        ws = torch.zeros(group_ws_bytes(probs, splits) // 4 + 1, device=DEV)
        tickets = torch.zeros(1024, dtype=torch.int32, device=DEV)
        gemm_group(probs, splits, ws, tickets)
        torch.cuda.synchronize()
        for p, r in zip(probs, refs):
            assert _rel(p.c, r) < 2e-5


@pytest.mark.parametrize("splits", [[3, 3, 3, 1], [4, 2, 1, 2]])
def test_gemm_sp_item_orders_agree(splits):
    """The fused split GEMM's two item orders (gemm_sp.hip g5_coords: tile-major, and the
    K-split-major default) on the paper group's shapes: fp32-accurate and bitwise equal (the
    split-K reduction sums the partial slabs in K order whatever order the items ran in)."""
    from pytorch_r2d2_amd.ops._lib import kernels
    from pytorch_r2d2_amd.ops.gemm import gemm_sp
    g = torch.Generator(device=DEV).manual_seed(11)
    probs, refs = [], []
    for (M, N, K, ak) in [(1024, 1568, 2560, 0), (1024, 256, 2560, 0), (512, 256, 2560, 0),
                          (2560, 1568, 1024, 1)]:
        x = _op(M, K, 1, g) if ak else _op(K, M, 1, g).t()
        y = _op(N, K, 0, g).t().contiguous()
        xh, xl = _split(x)
        yh, yl = _split(y)
        probs.append(Gemm(xh, yh, torch.zeros(M, N, device=DEV), a_lo=xl, b_lo=yl))
        refs.append(x.double() @ y.double())
    k = kernels()
    outs = {}
    try:
        for mode in (1 | 64, 1):                 # bit 6: tile-major; default: K-split-major
            k.r2_gemm5_set_mode(mode)
            for p in probs:
                p.c.zero_()
            gemm_sp(probs, splits=splits, cfg=6)
            torch.cuda.synchronize()
            outs[mode] = [p.c.clone() for p in probs]
    finally:
        k.r2_gemm5_set_mode(1)
    for a, b, r in zip(outs[1 | 64], outs[1], refs):
        assert torch.equal(a, b)
        assert _rel(b, r) < 2e-5


def _make(mode, B=16, preset="atari57", dtype="fp32", **kw):
    from pytorch_r2d2_amd.config import get_config
    from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    from pytorch_r2d2_amd.models import QNet
    over = {"learner.batch_size": B, "learner.target_mode": mode, "replay.capacity": 40000,
            "replay.n_subrings": 8, "learner.use_graph": False, "learner.compute_dtype": dtype,
            "replay.burn_in": 6, "replay.learn": 8, "replay.overlap": 7}
    over.update(kw)
    cfg = get_config(preset, **over)
    rp = HBMReplay(cfg, DEV)
    rp.fill_synthetic(episode_len=100, seed=5)
    torch.manual_seed(7)
    net = QNet("cpu", cfg.model, cfg.env)
    tgt = QNet("cpu", cfg.model, cfg.env)
    eng = LearnerEngine(cfg, rp, DEV, init_module=net)
    eng.layout.load_state_dict(eng.target, tgt.state_dict())
    eng._pack(always=True)
    return cfg, rp, eng, net, tgt


def _oracle(rp, eng, net, tgt, cfg, mode, dtype=torch.float64):
    """Autograd oracle of the same batch on the CPU (exact IEEE arithmetic, no library fast paths)
    in ``dtype``: float64 = the truth, float32 = what a plain fp32 PyTorch learner computes."""
    from pytorch_r2d2_amd.learner_ref import batch_from_hbm, r2d2_loss
    online = copy.deepcopy(net).to(dtype)
    target = copy.deepcopy(tgt).to(dtype)
    batch = batch_from_hbm(rp, eng.starts, eng.probs, cfg, "cpu")
    for f in ("obs", "h0", "c0", "th0", "tc0", "nh0", "nc0", "reward", "done", "weights"):
        v = getattr(batch, f)
        if v is not None:
            setattr(batch, f, v.to(dtype))
    out = r2d2_loss(online, target, batch, cfg, mode)
    out["loss"].backward()
    return online, out


def _oracle64(rp, eng, net, tgt, cfg, mode):
    return _oracle(rp, eng, net, tgt, cfg, mode, torch.float64)


# "" = the defaults (dh = dz . W1 inside the BPTT, learner.bptt_dh); "nodh": dh on the TD
# launch's MFMAs (learner.td_fuse_dh).  (Round 5's GEMMs on the BPTT's helper workgroups were
# removed with their oracle cases: profiles/r05_bptt_helpers_roles.txt.)
_FUSED = {"": {}, "nodh": {"learner.bptt_dh": False}}


@pytest.mark.parametrize("mode,preset,fused", [("fixed", "atari57", ""), ("shifted", "atari57", ""),
                                               ("reference", "atari57", ""), ("fixed", "dmlab30", ""),
                                               ("fixed", "atari57", "nodh")])
def test_engine_fp32_matches_fp64_oracle(mode, preset, fused):
    """The fp32 (split-precision) learner step against the float64 truth, with plain fp32 PyTorch
    as the yardstick.  With random-init nets the TD error is a small difference of two Q values,
    so every fp32 implementation's gradient error is amplified: fp32 PyTorch itself lands 1e-4 ..
    5e-4 off float64 on these tensors (tools/sp_oracle_calib.py, CPU and GPU alike).  The engine
    must be within 1e-4 of the truth or no worse than 2x fp32 PyTorch, on the loss, all 18
    gradients and the replay priorities; its forward activations are ~5e-6 off (test below).
    dmlab30 (RGB 3x72x96): the fp32 library torso (ops/torso_lib.py) feeding the split planes."""
    cfg, rp, eng, net, tgt = _make(mode, preset=preset, **_FUSED[fused])
    assert eng.sp_lib == (preset == "dmlab30")
    eng._forward_loss()
    eng._backward_core()
    eng._backward_torso()
    torch.cuda.synchronize()
    assert eng.error_word() == 0
    online, out = _oracle64(rp, eng, net, tgt, cfg, mode)
    on32, out32 = _oracle(rp, eng, net, tgt, cfg, mode, torch.float32)
    l64 = out["loss"].item()
    lrel = abs(eng.loss.item() - l64) / l64
    lrel32 = abs(out32["loss"].item() - l64) / l64
    got = eng.layout.views(eng.grad)
    g32 = dict(on32.named_parameters())
    errs = {n: (_rel(got[n].cpu(), p.grad), _rel(g32[n].grad, p.grad)) for n, p in online.named_parameters()}
    assert lrel < max(1e-4, 2 * lrel32), (lrel, lrel32)
    bad = {k: v for k, v in errs.items() if v[0] > max(1e-4, 2 * v[1])}
    assert not bad, errs
    Lb, T = cfg.replay.burn_in, cfg.replay.seq_len
    s = eng.starts.long()
    base = s - s % rp.cap_e
    rows = base[None] + (s[None] - base[None] + torch.arange(Lb, T, device=DEV)[:, None]) % rp.cap_e
    p32 = _rel(out32["priority"], out["priority"])
    assert _rel(rp.priority[rows].cpu(), out["priority"]) < max(1e-4, 2 * p32)
    if preset == "dmlab30":     # the library convs inside the captured step
        eng.capture(warmup=1)
        for _ in range(3):
            eng.step()
        torch.cuda.synchronize()
        assert eng.error_word() == 0 and torch.isfinite(eng.master).all()


@pytest.mark.parametrize("bptt", ["", "nodh"])
def test_engine_fp32_matches_fp64_oracle_at_bench_shape(bptt):
    """The benched step itself (atari57: B=64, burn-in 40 + learn 40, n=5, fixed target) against
    the float64 truth: the 12 LSTM groups (3 chains x 4 batch tiles) placed two per XCD, the
    85-step tagged T4 hand-offs (the 4-bit tags wrap 5 times per launch), the 192x256 split GEMM
    tiles, the full-chip torso grids.  Same bounds as the reduced-shape test; then 5 replays of
    the captured (hoisted) graphs with the persistent kernels' error word still 0.  Default: the
    BPTT computes its input gradient dz . W1 itself (learner.bptt_dh); ``nodh``: the TD launch
    does."""
    over = {"replay.burn_in": 40, "replay.learn": 40, "replay.overlap": 40, "replay.n_step": 5,
            "replay.capacity": 64000}
    over.update(_FUSED[bptt])
    cfg, rp, eng, net, tgt = _make("fixed", B=64, **over)
    assert (eng.B, eng.Lb, eng.Ll, eng.n, eng.Tn) == (64, 40, 40, 5, 85)
    rp.fill_synthetic(episode_len=200, seed=5)
    eng._forward_loss()
    eng._backward_core()
    eng._backward_torso()
    torch.cuda.synchronize()
    assert eng.error_word() == 0
    online, out = _oracle64(rp, eng, net, tgt, cfg, "fixed")
    on32, out32 = _oracle(rp, eng, net, tgt, cfg, "fixed", torch.float32)
    l64 = out["loss"].item()
    lrel = abs(eng.loss.item() - l64) / l64
    lrel32 = abs(out32["loss"].item() - l64) / l64
    assert lrel < max(1e-4, 2 * lrel32), (lrel, lrel32)
    got = eng.layout.views(eng.grad)
    g32 = dict(on32.named_parameters())
    errs = {n: (_rel(got[n].cpu(), p.grad), _rel(g32[n].grad, p.grad)) for n, p in online.named_parameters()}
    assert len(errs) == 18
    bad = {k: v for k, v in errs.items() if v[0] > max(1e-4, 2 * v[1])}
    assert not bad, errs
    Lb, T = cfg.replay.burn_in, cfg.replay.seq_len
    s = eng.starts.long()
    base = s - s % rp.cap_e
    rows = base[None] + (s[None] - base[None] + torch.arange(Lb, T, device=DEV)[:, None]) % rp.cap_e
    p32 = _rel(out32["priority"], out["priority"])
    assert _rel(rp.priority[rows].cpu(), out["priority"]) < max(1e-4, 2 * p32)
    eng.capture(warmup=1)
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize()
    assert eng.error_word() == 0
    assert torch.isfinite(eng.master).all() and torch.isfinite(eng.loss).all()


def test_engine_fp32_forward_activations():
    """Torso features, x-projection, recurrent states and Q values of the fp32 engine vs float64:
    <= 2e-5 relative (bf16: ~3e-3)."""
    from pytorch_r2d2_amd.learner_ref import batch_from_hbm
    cfg, rp, eng, net, tgt = _make("fixed")
    eng._forward_loss()
    torch.cuda.synchronize()
    on = net.double()
    b = batch_from_hbm(rp, eng.starts, eng.probs, cfg, "cpu")
    obs = b.obs.double()
    Tn, B = obs.shape[:2]
    T, Lb = cfg.replay.seq_len, cfg.replay.burn_in
    with torch.no_grad():
        X = on.torso(obs.reshape(Tn * B, *obs.shape[2:]))
        assert _rel(eng.X_on.cpu().double() + eng.X_on_lo.cpu().double(), X) < 2e-5
        xp = X @ on.lstm.weight_ih.t() + on.lstm.bias_ih + on.lstm.bias_hh
        assert _rel(eng.xp_on.cpu().double(), xp[:, eng.layout.gate_perm]) < 2e-5
        hs, cs = on.lstm_seq(X.reshape(Tn, B, -1)[:T], b.h0.double(), b.c0.double())
        he = eng.hseq["on"].cpu().double() + eng.hseq_lo["on"].cpu().double()
        assert _rel(he, hs) < 2e-5 and _rel(eng.cseq["on"].cpu().double(), cs) < 2e-5
        q = on.head(hs[Lb:]).reshape(-1, cfg.model.n_actions)
        assert _rel(eng.q_on.cpu().double(), q) < 2e-5


def test_engine_fp32_is_closer_to_oracle_than_bf16():
    """The same step in bf16 is ~1e-2 off the fp64 oracle; fp32 (split) must be >= 50x closer."""
    res = {}
    for dt in ("bf16", "fp32"):
        cfg, rp, eng, net, tgt = _make("fixed", dtype=dt)
        eng._forward_loss()
        eng._backward_core()
        eng._backward_torso()
        torch.cuda.synchronize()
        online, out = _oracle64(rp, eng, net, tgt, cfg, "fixed")
        got = eng.layout.views(eng.grad)
        res[dt] = max(_rel(got[n].cpu(), p.grad) for n, p in online.named_parameters())
    assert res["fp32"] * 50 < res["bf16"], res


def test_engine_fp32_graph_step_and_seaquest_actions():
    """fp32 engine: graph capture replays the eager step; an 18-action head (Seaquest) runs the
    fused TD/head path (no torch.mm fallback) and matches the oracle."""
    cfg, rp, eng, net, tgt = _make("fixed", B=16, preset="seaquest8")
    assert eng.layout.A == 18
    eng._forward_loss()
    eng._backward_core()
    eng._backward_torso()
    torch.cuda.synchronize()
    online, out = _oracle64(rp, eng, net, tgt, cfg, "fixed")
    on32, _ = _oracle(rp, eng, net, tgt, cfg, "fixed", torch.float32)
    got = eng.layout.views(eng.grad)
    g32 = dict(on32.named_parameters())
    errs = {n: (_rel(got[n].cpu(), p.grad), _rel(g32[n].grad, p.grad)) for n, p in online.named_parameters()}
    assert all(e <= max(1e-4, 2 * e32) for e, e32 in errs.values()), errs
    cfg2, rp2, eng2, _, _ = _make("fixed", B=16)
    cfg3, rp3, eng3, _, _ = _make("fixed", B=16)
    for _ in range(2):
        eng2.step_eager()
    eng3.capture(warmup=0)
    eng3.step()
    eng3.step()
    torch.cuda.synchronize()
    assert torch.equal(rp2.step, rp3.step)
    assert _rel(eng3.master, eng2.master) < 1e-6
    assert eng3.error_word() == 0


def test_torso_fwd_sp_matches_fp64():
    """torso_fwd_sp2_kernel (int8-digit conv1, split conv2 / conv3) over 4 jobs with uneven frame
    counts (partial last rounds of the grid-stride loop) and activation saves, against a float64
    conv stack of the same split weights (w = hi + lo): features and the saved channels-last act1 /
    act2 planes to fp32 accuracy."""
    import numpy as np
    import torch.nn.functional as F
    from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle
    k = kernels()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    cap = 3000
    frames = torch.randint(0, 256, (cap, 4 * 84 * 84), dtype=torch.uint8, device=dev, generator=g)
    counts = [301, 517, 45, 260]
    rows = [torch.randint(0, cap, (n,), dtype=torch.int32, device=dev, generator=g) for n in counts]

    def net():
        w = [_split(torch.randn(32, kk, device=dev, generator=g) * 0.05) for kk in (256, 512, 288)]
        b = [torch.randn(32, device=dev, generator=g) * 0.1 for _ in range(3)]
        return w, b

    nets = [net(), net()]
    outs, jobs = [], []
    for j, n in enumerate(counts):
        (w, b) = nets[j == 3]
        X = torch.full((2, n, 1568), 7.0, dtype=torch.bfloat16, device=dev)
        save = j == 1
        s1 = torch.zeros(2, n, 400, 32, dtype=torch.bfloat16, device=dev) if save else None
        s2 = torch.zeros(2, n, 81, 32, dtype=torch.bfloat16, device=dev) if save else None
        outs.append((X, s1, s2))
        jobs.append([ptr(rows[j]), n, ptr(w[0][0]), ptr(w[0][1]), ptr(b[0]), ptr(w[1][0]),
                     ptr(w[1][1]), ptr(b[1]), ptr(w[2][0]), ptr(w[2][1]), ptr(b[2]), ptr(X[0]),
                     ptr(X[1]), ptr(s1[0]) if save else 0, ptr(s1[1]) if save else 0,
                     ptr(s2[0]) if save else 0, ptr(s2[1]) if save else 0, 0, 0, 0])
    arr = np.asarray(jobs, dtype=np.int64)
    n_cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert k.r2_torso_fwd_sp_multi(ptr(frames), arr.ctypes.data, len(jobs), n_cus, stream_handle()) == 0
    torch.cuda.synchronize()
    both = lambda x: x[0].double() + x[1].double()   # noqa: E731
    for j, (X, s1, s2) in enumerate(outs):
        (w, b) = nets[j == 3]
        wd = [(hi.double() + lo.double()) for hi, lo in w]
        # kernel weight layouts (engine/layout.py): conv1 K = (by, bx, ci, dy, dx) with kh = 4 by +
        # dy, kw = 4 bx + dx (space-to-depth), conv2 / conv3 (kh, kw, ci)
        W1 = wd[0].view(32, 2, 2, 4, 4, 4).permute(0, 3, 1, 4, 2, 5).reshape(32, 4, 8, 8)
        W2 = wd[1].view(32, 4, 4, 32).permute(0, 3, 1, 2)
        W3 = wd[2].view(32, 3, 3, 32).permute(0, 3, 1, 2)
        x = frames[rows[j].long()].double().view(-1, 4, 84, 84) / 255.0   # the kernel's /255 input scale
        a1 = F.relu(F.conv2d(x, W1, b[0].double(), stride=4))
        a2 = F.relu(F.conv2d(a1, W2, b[1].double(), stride=2))
        a3 = F.relu(F.conv2d(a2, W3, b[2].double(), stride=1))
        assert not (X == 7.0).any()
        assert _rel(both(X), a3.reshape(a3.shape[0], -1)) < 2e-5
        if s1 is not None:
            assert _rel(both(s1), a1.permute(0, 2, 3, 1).reshape(-1, 400, 32)) < 2e-5
            assert _rel(both(s2), a2.permute(0, 2, 3, 1).reshape(-1, 81, 32)) < 2e-5


def test_td_fused_dh_matches_fp64_split():
    """Split precision: the fused dh (3 MFMA passes over dz / W1^T hi-lo planes) vs float64 of the
    same split operands: fp32-accurate.  (learner.bptt_dh off: by default the BPTT computes dh
    itself, covered by the engine oracles through every BPTT gradient.)"""
    cfg, rp, eng, net, tgt = _make("fixed", **{"learner.bptt_dh": False})
    eng._forward_loss()
    torch.cuda.synchronize()
    assert eng._dh_done
    N = eng.Ll * eng.B
    dz = eng.dz[:N].double() + eng.dz_lo[:N].double()
    w1 = eng.pk["head1"].double() + eng.pk_lo["head1"].double()
    assert _rel(eng.dh[:N], dz @ w1) < 2e-5


@pytest.mark.parametrize("fill", [0, -1])
def test_lstm_sp_tagged_word_handoff_over_launches(fill):
    """The split-precision LSTM forward's 4-byte tagged-word hand-off (lstm_persist.hip T4: 4-bit
    {epoch parity, step} tags) over 5 consecutive launches on ONE ring + ctr with different inputs
    each time (stale words of the previous launch must never be taken), on a zero- and a
    (-1)-filled ring, against a float64 recurrence.  (The 8-byte {h, tag} granule form it was
    first checked against was removed in round 6.)"""
    import numpy as np
    from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle
    k = kernels()
    H, B, T, NC = 256, 64, 23, 3
    G = 4 * H
    g = torch.Generator(device=DEV).manual_seed(3)
    nwg = H // 16
    whh = torch.randn(nwg, 64, H, device=DEV, generator=g) * 0.06
    wh, wl = _split(whh)
    c0 = torch.randn(B, H, device=DEV, generator=g) * 0.5
    h0 = torch.randn(B, H, device=DEV, generator=g) * 0.5
    err = torch.zeros(1, dtype=torch.int32, device=DEV)

    def site():
        return (torch.zeros(int(k.r2_lstm_persist_ctr_words()), dtype=torch.int32, device=DEV),
                torch.full((k.r2_lstm_tag_ring_bytes(4, B, H) // 4,), fill, dtype=torch.int32,
                           device=DEV))

    outs = {}
    for name, (ctr, ring) in (("t4", site()),):
        res = []
        for launch in range(5):
            xp = torch.randn(T * B, G, device=DEV, generator=torch.Generator(device=DEV).manual_seed(launch))
            bufs, desc = [], []
            for _ in range(NC):
                hs = torch.zeros(T, B, H, dtype=torch.bfloat16, device=DEV)
                hl, cs = torch.zeros_like(hs), torch.zeros(T, B, H, device=DEV)
                bufs.append((hs, hl, cs))
                desc += [ptr(xp), ptr(wh), ptr(h0), ptr(c0), ptr(hs), ptr(cs), 0, 0, 0, ptr(wl), ptr(hl)]
            arr = np.asarray(desc, dtype=np.int64)
            rc = k.r2_lstm_fwd_tag_sp(arr.ctypes.data, NC, B, T, H, ptr(ctr), ptr(err), ptr(ring),
                                      stream_handle())
            assert rc == 0
            torch.cuda.synchronize()
            assert err.item() == 0
            res.append((xp, bufs))
        outs[name] = res
    # float64 recurrence (packed gate layout: workgroup j owns units 16j..16j+15, gate-major rows)
    W = whh.double().view(nwg, 4, 16, H)                      # [j][gate][unit][k]
    for xp, b4 in outs["t4"]:
        h, c = h0.double(), c0.double()
        x = xp.double().view(T, B, nwg, 4, 16)
        for t in range(T):
            gt = torch.einsum("bk,jguk->bjgu", h, W) + x[t]
            i_, f_, gg, o_ = (gt[:, :, q] for q in range(4))
            c = torch.sigmoid(f_) * c.view(B, nwg, 16) + torch.sigmoid(i_) * torch.tanh(gg)
            h = torch.sigmoid(o_) * torch.tanh(c)
            c, h = c.reshape(B, H), h.reshape(B, H)
            for hs, hl, cs in b4:
                h4 = hs[t].double() + hl[t].double()
                assert _rel(h4, h) < 2e-5, t
                assert _rel(cs[t], c) < 2e-5, t
