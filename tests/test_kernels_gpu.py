"""Numerics of every HIP kernel against a plain fp32 PyTorch reference of the same op."""
import numpy as np
import pytest
import torch

from pytorch_r2d2_amd.config import get_config
from pytorch_r2d2_amd.engine.layout import ParamLayout, UNITS
from pytorch_r2d2_amd.models import QNet
from pytorch_r2d2_amd.ops._lib import kernels, ptr, stream_handle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _setup(B=8, H=256, seed=0, preset="atari57"):
    cfg = get_config(preset, **{"model.hidden": H})
    torch.manual_seed(seed)
    net = QNet("cpu", cfg.model, cfg.env)
    L = ParamLayout(cfg.model, cfg.env)
    flat = L.from_module(net, DEV)
    bf = torch.zeros(L.bf_numel, dtype=torch.bfloat16, device=DEV)
    f32 = torch.zeros(L.f_numel, device=DEV)
    k = kernels()
    k.r2_pack_bf16(ptr(flat), ptr(L.bf_index.to(DEV)), ptr(bf), L.bf_numel, stream_handle())
    k.r2_gather_f32(ptr(flat), ptr(L.f_index.to(DEV)), ptr(f32), L.f_numel, stream_handle())
    return cfg, net.to(DEV), L, flat, L.packed_views(bf, f32)


@pytest.mark.parametrize("impl", ["step", "persistent", "tagged"])
@pytest.mark.parametrize("B,H", [(8, 256), (64, 256), (40, 128), (128, 256), (16, 512), (33, 64)])
def test_lstm_forward_matches_lstmcell(B, H, impl):
    cfg, net, L, flat, pk = _setup(B, H)
    T = 7
    G = 4 * H
    x = torch.randn(T, B, L.D, device=DEV) * 0.5
    h0 = torch.randn(B, H, device=DEV) * 0.3
    c0 = torch.randn(B, H, device=DEV) * 0.3
    # reference in fp32 with bf16-rounded inputs/weights (the kernel's operand precision)
    xb = x.bfloat16().float()
    wih = net.lstm.weight_ih.bfloat16().float()
    whh = net.lstm.weight_hh.bfloat16().float()
    b = net.lstm.bias_ih + net.lstm.bias_hh
    h, c = h0.bfloat16().float(), c0.clone()
    ref_h, ref_c = [], []
    for t in range(T):
        g = xb[t] @ wih.t() + b + h.bfloat16().float() @ whh.t()
        i, f, gg, o = g.chunk(4, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        ref_h.append(h)
        ref_c.append(c)
    ref_h, ref_c = torch.stack(ref_h), torch.stack(ref_c)
    perm = L.gate_perm.to(DEV)
    xproj = (xb.view(T * B, -1) @ wih[perm].t() + b[perm]).contiguous()
    hseq = torch.zeros(T, B, H, dtype=torch.bfloat16, device=DEV)
    cseq = torch.zeros(T, B, H, device=DEV)
    h32 = torch.zeros(T, B, H, device=DEV)
    gates = torch.zeros(T, B, G, device=DEV)
    h0b = h0.bfloat16()
    chain = [ptr(xproj), ptr(pk["w_hh"]), ptr(h0b), ptr(c0), ptr(hseq), ptr(cseq), ptr(h32),
             ptr(gates), 0]
    arr = np.asarray(chain * 2, dtype=np.int64)  # two identical chains in one launch
    hseq2 = torch.zeros_like(hseq)
    cseq2 = torch.zeros_like(cseq)
    arr[9 + 4] = ptr(hseq2)
    arr[9 + 5] = ptr(cseq2)
    arr[9 + 6] = 0
    arr[9 + 7] = 0
    if impl == "step":
        rc = kernels().r2_lstm_fwd(arr.ctypes.data, 2, B, T, H, 0, stream_handle())
    else:
        ctr = torch.zeros(int(kernels().r2_lstm_persist_ctr_words()), dtype=torch.int32, device=DEV)
        err = torch.zeros(1, dtype=torch.int32, device=DEV)
        if impl == "tagged":
            ring = torch.full((kernels().r2_lstm_tag_ring_bytes(2, B, H) // 4,), -1,
                              dtype=torch.int32, device=DEV)   # garbage content is fine
            rc = kernels().r2_lstm_fwd_tag(arr.ctypes.data, 2, B, T, H, ptr(ctr), ptr(err),
                                           ptr(ring), stream_handle())
        else:
            rc = kernels().r2_lstm_fwd_persist(arr.ctypes.data, 2, B, T, H, ptr(ctr), ptr(err),
                                               stream_handle())
    assert rc == 0
    if impl != "step":
        torch.cuda.synchronize()
        assert err.item() == 0
    torch.cuda.synchronize()
    assert _rel(h32, ref_h) < 2e-2
    assert _rel(cseq, ref_c) < 2e-2
    assert torch.equal(cseq, cseq2)
    # saved gates (packed) == activations of the reference gate pre-activations
    g_last = (xb[-1] @ wih.t() + b + ref_h[-2].bfloat16().float() @ whh.t())
    act = torch.cat([torch.sigmoid(g_last[:, :2 * H]), torch.tanh(g_last[:, 2 * H:3 * H]),
                     torch.sigmoid(g_last[:, 3 * H:])], 1)
    assert _rel(gates[-1], act[:, perm]) < 3e-2


@pytest.mark.parametrize("impl", ["step", "persistent", "tagged"])
@pytest.mark.parametrize("B,H", [(8, 256), (64, 256), (96, 128), (16, 512), (33, 64)])
def test_lstm_backward_matches_autograd(B, H, impl):
    cfg, net, L, flat, pk = _setup(B, H, seed=1)
    T, t0 = 9, 3
    G = 4 * H
    x = (torch.randn(T, B, L.D, device=DEV) * 0.5).bfloat16().float()
    h0 = (torch.randn(B, H, device=DEV) * 0.3).bfloat16().float()
    c0 = torch.randn(B, H, device=DEV) * 0.3
    perm = L.gate_perm.to(DEV)
    wih = net.lstm.weight_ih.detach().bfloat16().float()
    whh = net.lstm.weight_hh.detach().bfloat16().float()
    b = (net.lstm.bias_ih + net.lstm.bias_hh).detach()
    xproj = (x.view(T * B, -1) @ wih[perm].t() + b[perm]).contiguous()
    hseq = torch.zeros(T, B, H, dtype=torch.bfloat16, device=DEV)
    cseq = torch.zeros(T, B, H, device=DEV)
    gates = torch.zeros(T - t0, B, G, device=DEV)
    h0b = h0.bfloat16()
    arr = np.asarray([ptr(xproj), ptr(pk["w_hh"]), ptr(h0b), ptr(c0), ptr(hseq), ptr(cseq), 0,
                      ptr(gates), t0], dtype=np.int64)
    k = kernels()
    assert k.r2_lstm_fwd(arr.ctypes.data, 1, B, T, H, 0, stream_handle()) == 0
    dh_ext = torch.randn(T - t0, B, H, device=DEV)
    nwg = H // UNITS
    s0 = torch.zeros(nwg, B, H, device=DEV)
    s1 = torch.zeros_like(s0)
    dc = torch.zeros(B, H, device=DEV)
    dg = torch.zeros(T - t0, B, G, dtype=torch.bfloat16, device=DEV)
    if impl == "step":
        assert k.r2_lstm_bwd(ptr(dh_ext), ptr(gates), ptr(cseq), ptr(c0), ptr(pk["w_hhT"]), ptr(s0),
                             ptr(s1), ptr(dc), ptr(dg), B, T, t0, H, stream_handle()) == 0
    elif impl == "tagged":
        ctr = torch.zeros(int(kernels().r2_lstm_persist_ctr_words()), dtype=torch.int32, device=DEV)
        err = torch.zeros(1, dtype=torch.int32, device=DEV)
        ring = torch.full((k.r2_lstm_bwd_tag_ring_bytes(B, H) // 4,), -1, dtype=torch.int32,
                          device=DEV)
        bias_ws = torch.zeros((B + 15) // 16, G, device=DEV)
        db1 = torch.full((G,), float("nan"), device=DEV)
        db2 = torch.full((G,), float("nan"), device=DEV)
        perm_i = L.gate_perm.to(DEV, torch.int32)
        for _ in range(2):      # second launch: stale granules of the first must be ignored
            assert k.r2_lstm_bwd_tag(ptr(dh_ext), ptr(gates), ptr(cseq), ptr(c0), ptr(pk["w_hhT"]),
                                     ptr(dg), B, T, t0, H, ptr(ctr), ptr(err), ptr(ring),
                                     ptr(bias_ws), ptr(perm_i), ptr(db1), ptr(db2), *([0] * 11),
                                     stream_handle()) == 0
        rest = ctr.clone()
        rest[3072 + 32] = rest[3072 + 64] = 0        # the two launch epochs (lstm_persist.hip PT_EPOCH_*)
        assert int(rest.abs().sum().item()) == 0      # counters self-reset by the last workgroup
    else:
        slab = torch.zeros(2, nwg, B, H, device=DEV)
        ctr = torch.zeros(int(kernels().r2_lstm_persist_ctr_words()), dtype=torch.int32, device=DEV)
        err = torch.zeros(1, dtype=torch.int32, device=DEV)
        assert k.r2_lstm_bwd_persist(ptr(dh_ext), ptr(gates), ptr(cseq), ptr(c0), ptr(pk["w_hhT"]),
                                     ptr(slab), ptr(dg), B, T, t0, H, ptr(ctr), ptr(err),
                                     stream_handle()) == 0
    torch.cuda.synchronize()
    if impl != "step":
        assert err.item() == 0
    # autograd reference: state after burn-in steps [0,t0) is a constant (detached)
    h, c = h0, c0
    with torch.no_grad():
        for t in range(t0):
            g = x[t] @ wih.t() + b + h @ whh.t()
            i, f, gg, o = g.chunk(4, 1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h = torch.sigmoid(o) * torch.tanh(c)
    pre, hs = [], []
    for t in range(t0, T):
        g = x[t] @ wih.t() + b + h @ whh.t()
        if not g.requires_grad:
            g.requires_grad_(True)
        else:
            g.retain_grad()
        pre.append(g)
        i, f, gg, o = g.chunk(4, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        hs.append(h)
    loss = sum((hh * dh_ext[i]).sum() for i, hh in enumerate(hs))
    loss.backward()
    ref = torch.stack([p.grad for p in pre])  # (T-t0, B, G) original gate order
    got = dg.float()[..., L.gate_inv.to(DEV)]
    assert _rel(got, ref) < 3e-2, [round(_rel(got[i], ref[i]), 4) for i in range(T - t0)]
    if impl == "tagged":   # fused bias gradient (fp32 column sums of dgates, torch gate order)
        assert _rel(db1, ref.sum((0, 1))) < 1e-2 and torch.equal(db1, db2)


@pytest.mark.parametrize("B", [64, 200])
def test_lstm_persistent_same_xcd_path_matches_sc1_path(B):
    """The same-XCD plain-store hand-off and the placement-independent sc1 hand-off must give
    bit-identical results (only the store flavour of the published h / dh partials differs)."""
    cfg, net, L, flat, pk = _setup(B, 256, seed=2)
    H, G, T, t0 = 256, 1024, 12, 4
    k = kernels()
    xproj = torch.randn(T * B, G, device=DEV)
    h0 = (torch.randn(B, H, device=DEV) * 0.3).bfloat16()
    c0 = torch.randn(B, H, device=DEV) * 0.3
    dh_ext = torch.randn(T - t0, B, H, device=DEV)
    nw = int(k.r2_lstm_persist_ctr_words())
    outs = []
    for slow in (0, 1):
        k.r2_lstm_persist_force_slow(slow)
        hseq = torch.zeros(T, B, H, dtype=torch.bfloat16, device=DEV)
        cseq = torch.zeros(T, B, H, device=DEV)
        gates = torch.zeros(T - t0, B, G, device=DEV)
        arr = np.asarray([ptr(xproj), ptr(pk["w_hh"]), ptr(h0), ptr(c0), ptr(hseq), ptr(cseq), 0,
                          ptr(gates), t0] * 2, dtype=np.int64)
        ctr = torch.zeros(nw, dtype=torch.int32, device=DEV)
        err = torch.zeros(1, dtype=torch.int32, device=DEV)
        assert k.r2_lstm_fwd_persist(arr.ctypes.data, 2, B, T, H, ptr(ctr), ptr(err), stream_handle()) == 0
        slab = torch.zeros(2, H // UNITS, B, H, device=DEV)
        dg = torch.zeros(T - t0, B, G, dtype=torch.bfloat16, device=DEV)
        assert k.r2_lstm_bwd_persist(ptr(dh_ext), ptr(gates), ptr(cseq), ptr(c0), ptr(pk["w_hhT"]),
                                     ptr(slab), ptr(dg), B, T, t0, H, ptr(ctr), ptr(err),
                                     stream_handle()) == 0
        torch.cuda.synchronize()
        assert err.item() == 0
        outs.append((hseq, cseq, dg))
    k.r2_lstm_persist_force_slow(0)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [64, 24])
def test_lstm_tagged_repeated_launches_and_placement(B):
    """Tagged forward hand-off: (1) granules left in the ring by earlier launches are never
    accepted (epoch tags): back-to-back launches with different inputs each match the counter
    kernel; (2) the same-XCD plain-store path and the sc1 path are bit-identical."""
    cfg, net, L, flat, pk = _setup(B, 256, seed=3)
    H, G, T = 256, 1024, 10
    k = kernels()
    nw = int(k.r2_lstm_persist_ctr_words())
    ctr = torch.zeros(nw, dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    ring = torch.zeros(k.r2_lstm_tag_ring_bytes(2, B, H) // 4, dtype=torch.int32, device=DEV)
    h0 = (torch.randn(B, H, device=DEV) * 0.3).bfloat16()
    c0 = torch.randn(B, H, device=DEV) * 0.3

    def run(fn_name, xproj, slow=0):
        k.r2_lstm_persist_force_slow(slow)
        hseq = torch.zeros(T, B, H, dtype=torch.bfloat16, device=DEV)
        cseq = torch.zeros(T, B, H, device=DEV)
        arr = np.asarray([ptr(xproj), ptr(pk["w_hh"]), ptr(h0), ptr(c0), ptr(hseq), ptr(cseq), 0,
                          0, 0] * 2, dtype=np.int64)
        if fn_name == "tag":
            rc = k.r2_lstm_fwd_tag(arr.ctypes.data, 2, B, T, H, ptr(ctr), ptr(err), ptr(ring),
                                   stream_handle())
        else:
            rc = k.r2_lstm_fwd_persist(arr.ctypes.data, 2, B, T, H, ptr(ctr), ptr(err),
                                       stream_handle())
        assert rc == 0
        torch.cuda.synchronize()
        k.r2_lstm_persist_force_slow(0)
        assert err.item() == 0
        return hseq, cseq

    for it in range(4):
        xproj = torch.randn(T * B, G, device=DEV) * (0.5 + it)
        h_t, c_t = run("tag", xproj, slow=it % 2)
        h_p, c_p = run("persist", xproj)
        assert _rel(c_t, c_p) < 1e-4, it
        assert _rel(h_t.float(), h_p.float()) < 1e-2, it
    xproj = torch.randn(T * B, G, device=DEV)
    a = run("tag", xproj, slow=0)
    b = run("tag", xproj, slow=1)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_lstm_tagged_three_chains_two_groups_per_xcd():
    """The fixed-target step's forward runs 3 chains x 4 batch tiles = 12 groups: placed two per
    XCD (lstm_persist.hip pl_decode map 2) every group takes the same-XCD hand-off; results are
    bit-identical to the spread placement and to the sc1 protocol, and match the counter kernel."""
    B, H, G, T = 64, 256, 1024, 9
    cfg, net, L, flat, pk = _setup(B, H, seed=5)
    k = kernels()
    nw = int(k.r2_lstm_persist_ctr_words())
    ctr = torch.zeros(nw, dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    ring = torch.zeros(k.r2_lstm_tag_ring_bytes(3, B, H) // 4, dtype=torch.int32, device=DEV)
    xps = [torch.randn(T * B, G, device=DEV) for _ in range(3)]
    h0s = [(torch.randn(B, H, device=DEV) * 0.3).bfloat16() for _ in range(3)]
    c0s = [torch.randn(B, H, device=DEV) * 0.3 for _ in range(3)]
    dbg = torch.zeros(1024, dtype=torch.int64, device=DEV)

    def run(fn_name, mode):
        k.r2_lstm_persist_force_slow(mode)
        outs, words = [], []
        for c in range(3):
            hs = torch.zeros(T, B, H, dtype=torch.bfloat16, device=DEV)
            cs = torch.zeros(T, B, H, device=DEV)
            outs.append((hs, cs))
            words += [ptr(xps[c]), ptr(pk["w_hh"]), ptr(h0s[c]), ptr(c0s[c]), ptr(hs), ptr(cs), 0, 0, 0]
        arr = np.asarray(words, dtype=np.int64)
        dbg.zero_()
        k.r2_lstm_persist_set_debug(ptr(dbg) if fn_name == "tag" else 0)
        if fn_name == "tag":
            rc = k.r2_lstm_fwd_tag(arr.ctypes.data, 3, B, T, H, ptr(ctr), ptr(err), ptr(ring),
                                   stream_handle())
        else:
            rc = k.r2_lstm_fwd_persist(arr.ctypes.data, 3, B, T, H, ptr(ctr), ptr(err),
                                       stream_handle())
        torch.cuda.synchronize()
        k.r2_lstm_persist_set_debug(0)
        k.r2_lstm_persist_force_slow(0)
        assert rc == 0 and err.item() == 0
        return outs, dbg[256:].cpu().clone()

    mapped, d = run("tag", 0)
    tags = [int(v) for v in d if v >= 1000]
    assert len(tags) == 12 * (H // UNITS)                      # every recurrence workgroup
    assert all(v % 10 == 1 for v in tags), "a group missed the same-XCD hand-off"
    spread, _ = run("tag", 2)
    sc1, _ = run("tag", 1)
    ref, _ = run("persist", 0)
    for c in range(3):
        for x, y, z in zip(mapped[c], spread[c], sc1[c]):
            assert torch.equal(x, y) and torch.equal(x, z), c
        assert _rel(mapped[c][1], ref[c][1]) < 1e-4
        assert _rel(mapped[c][0].float(), ref[c][0].float()) < 1e-2


def test_torso_matches_conv_stack():
    cfg, net, L, flat, pk = _setup()
    n = 37
    frames = torch.randint(0, 256, (50, 4 * 84 * 84), dtype=torch.uint8, device=DEV)
    rows = torch.randint(0, 50, (n,), dtype=torch.int32, device=DEV)
    out = torch.zeros(n, 1568, dtype=torch.bfloat16, device=DEV)
    a1 = torch.zeros(n, 400, 32, dtype=torch.bfloat16, device=DEV)
    a2 = torch.zeros(n, 81, 32, dtype=torch.bfloat16, device=DEV)
    for grid in (256, 5):  # one frame per block, and grid-stride with prefetch
        rc = kernels().r2_torso_fwd(ptr(frames), ptr(rows), n, ptr(pk["conv1"]), ptr(pk["b1"]),
                                    ptr(pk["conv2"]), ptr(pk["b2"]), ptr(pk["conv3"]), ptr(pk["b3"]),
                                    ptr(out), ptr(a1), ptr(a2), grid, stream_handle())
        assert rc == 0
        torch.cuda.synchronize()
        x = frames[rows.long()].view(n, 4, 84, 84).float() / 255.0
        with torch.no_grad():
            v = net.vis_layers
            r1 = torch.relu(v[0](x))
            r2 = torch.relu(v[2](r1))
            ref = torch.relu(v[4](r2)).reshape(n, -1)
        assert _rel(out, ref) < 2e-2
        assert _rel(a1.view(n, 20, 20, 32).permute(0, 3, 1, 2), r1) < 2e-2
        assert _rel(a2.view(n, 9, 9, 32).permute(0, 3, 1, 2), r2) < 2e-2


def test_torso_dmlab_rgb_matches_conv_stack():
    """The geometry-templated fused forward on DMLab-30 RGB frames (3x72x96 -> 32x17x23 ->
    32x7x10 -> 32x5x8) vs the fp32 PyTorch conv stack, with padded replay rows (row stride >
    frame bytes) and activation saves, several jobs in one launch."""
    import numpy as np
    from pytorch_r2d2_amd.ops.torso_lib import torso_fwd_fused
    cfg, net, L, flat, pk = _setup(preset="dmlab30")
    n0, n1 = 29, 18
    fb = 3 * 72 * 96
    store = torch.randint(0, 256, (60, fb + 64), dtype=torch.uint8, device=DEV)
    rows = torch.randint(0, 60, (n0 + n1,), dtype=torch.int32, device=DEV)
    out = torch.zeros(n0 + n1, 1280, dtype=torch.bfloat16, device=DEV)
    a1 = torch.zeros(n1, 391, 32, dtype=torch.bfloat16, device=DEV)
    a2 = torch.zeros(n1, 70, 32, dtype=torch.bfloat16, device=DEV)
    w = [ptr(pk[k]) for k in ("conv1", "b1", "conv2", "b2", "conv3", "b3")]
    for grid in (256, 7):
        jobs = np.asarray([[ptr(rows), n0, *w, ptr(out), 0, 0, 0],
                           [ptr(rows) + 4 * n0, n1, *w, ptr(out) + 2 * 1280 * n0, ptr(a1), ptr(a2), 0]],
                          dtype=np.int64)
        out.zero_()
        torso_fwd_fused(store, jobs, (3, 72, 96), grid)
        torch.cuda.synchronize()
        x = store[rows.long(), :fb].view(-1, 3, 72, 96).float() / 255.0
        with torch.no_grad():
            v = net.vis_layers
            r1 = torch.relu(v[0](x))
            r2 = torch.relu(v[2](r1))
            ref = torch.relu(v[4](r2)).reshape(n0 + n1, -1)
        assert _rel(out, ref) < 2e-2
        assert _rel(a1.view(n1, 17, 23, 32).permute(0, 3, 1, 2), r1[n0:]) < 2e-2
        assert _rel(a2.view(n1, 7, 10, 32).permute(0, 3, 1, 2), r2[n0:]) < 2e-2


def test_dueling_head_fwd_bwd():
    cfg, net, L, flat, pk = _setup()
    N, H, HD, A = 77, 256, 256, 6
    h = torch.randn(N, H, device=DEV).bfloat16()
    z = torch.mm(h, pk["head1"].t())
    q = torch.zeros(N, A, device=DEV)
    zr = torch.zeros(N, 2 * HD, dtype=torch.bfloat16, device=DEV)
    k = kernels()
    assert k.r2_dueling_fwd(ptr(z), ptr(pk["head_b1"]), ptr(pk["head_w2"]), ptr(pk["head_b2"]),
                            ptr(q), ptr(zr), N, A, HD, stream_handle()) == 0
    hf = h.float().requires_grad_(True)
    with torch.enable_grad():
        ref = net.head(hf)
    assert _rel(q, ref) < 2e-2
    dq = torch.randn(N, A, device=DEV)
    dz = torch.zeros(N, 2 * HD, dtype=torch.bfloat16, device=DEV)
    dva = torch.zeros(N, 1 + A, device=DEV)
    assert k.r2_dueling_bwd(ptr(dq), ptr(zr), ptr(pk["head_w2"]), ptr(dz), ptr(dva), N, A, HD,
                            stream_handle()) == 0
    dh = torch.mm(dz, pk["head1"]).float()
    ref.backward(dq)
    torch.cuda.synchronize()
    assert _rel(dh, hf.grad) < 3e-2
    g_v = torch.mm(dva.t(), zr.float())
    assert _rel(g_v[0, :HD], net.val[2].weight.grad[0]) < 3e-2
    assert _rel(g_v[1:, HD:], net.adv[2].weight.grad) < 3e-2


def test_rmsprop_centered_matches_torch():
    n = 100003
    p = torch.randn(n + 1, device=DEV)[:n].clone()  # odd size exercises the tail loop
    g = torch.randn(n, device=DEV)
    sq = torch.zeros(n, device=DEV)
    ga = torch.zeros(n, device=DEV)
    ref = p.clone().requires_grad_(True)
    opt = torch.optim.RMSprop([ref], lr=6.25e-5, alpha=0.95, eps=1.5e-7, centered=True)
    k = kernels()
    for _ in range(3):
        assert k.r2_rmsprop_centered(ptr(p), ptr(g), ptr(sq), ptr(ga), n, 6.25e-5, 0.95, 1.5e-7,
                                     1.0, 0, 0.0, stream_handle()) == 0
        ref.grad = g.clone()
        opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(p, ref.detach(), atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("sp,due", [(True, False), (True, True), (False, True)])
def test_rmsprop_pack_matches_update_then_gather(sp, due):
    """optim.hip rmsprop_pack_kernel (the update writes the LSTM / head row packs and, when due,
    the target master) + the prefix pack launch == rmsprop_centered + the full pack launch, bit
    for bit: master, optimizer state, online and target packs (hi and lo planes)."""
    cfg = get_config("atari57")
    L = ParamLayout(cfg.model, cfg.env)
    assert L.row_dst4 is not None
    n = L.padded
    torch.manual_seed(0)
    p0 = torch.randn(n, device=DEV) * 0.05
    g = torch.randn(n, device=DEV) * 1e-3
    sq0 = torch.rand(n, device=DEV) * 1e-6 + 1e-6
    ga0 = torch.randn(n, device=DEV) * 1e-5
    idx, fidx, dst4 = L.bf_index.to(DEV), L.f_index.to(DEV), L.row_dst4.to(DEV)
    nb = 2 * L.bf_numel if sp else L.bf_numel
    lo = L.bf_numel if sp else 0
    step = torch.tensor([1 if due else 0], dtype=torch.int64, device=DEV)   # interval 2
    k, s = kernels(), stream_handle()
    outs = []
    for fused in (False, True):
        p, sq, ga = p0.clone(), sq0.clone(), ga0.clone()
        tgt = torch.zeros(n, device=DEV)
        bf = torch.zeros(nb, dtype=torch.bfloat16, device=DEV)
        bft = torch.zeros(nb, dtype=torch.bfloat16, device=DEV)
        f32 = torch.zeros(L.f_numel, device=DEV)
        f32t = torch.zeros(L.f_numel, device=DEV)
        lb = torch.zeros(L.G, device=DEV)
        lbt = torch.zeros(L.G, device=DEV)
        if fused:
            assert k.r2_rmsprop_pack(ptr(p), ptr(g), ptr(sq), ptr(ga), n, 6.25e-5, 0.95, 1.5e-7, 1.0,
                                     0, 0.0, ptr(dst4), ptr(bf), ptr(bft), lo, ptr(tgt), ptr(step), 2,
                                     s) == 0
            n_master, n_bf = 0, L.bf_rows_begin
        else:
            assert k.r2_rmsprop_centered(ptr(p), ptr(g), ptr(sq), ptr(ga), n, 6.25e-5, 0.95, 1.5e-7,
                                         1.0, 0, 0.0, s) == 0
            n_master, n_bf = n, L.bf_numel
        assert k.r2_pack_step(ptr(p), ptr(tgt), n_master, ptr(idx), ptr(bf), ptr(bft), n_bf,
                              ptr(fidx), ptr(f32), ptr(f32t), L.f_numel, L.f_offsets["b_ih"][0],
                              L.f_offsets["b_hh"][0], ptr(lb), ptr(lbt), L.G, ptr(step), 2, lo,
                              s) == 0
        torch.cuda.synchronize()
        outs.append((p, sq, ga, tgt, bf, bft, f32, f32t, lb, lbt))
    # padding slots of the packs (no master element) are not written by the fused path
    real = torch.ones(L.bf_numel, dtype=torch.bool, device=DEV)
    real[L.bf_rows_begin:] = L.bf_index[L.bf_rows_begin:].to(DEV) != L.segs["lstm.bias_ih"].offset
    if sp:
        real = torch.cat([real, real])
    for name, a, b in zip(("p", "sq", "ga", "target", "bf", "bf_t", "f32", "f32_t", "lb", "lb_t"),
                          outs[0], outs[1]):
        if name in ("bf", "bf_t"):
            a, b = a[real], b[real]
        assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a,
                           b.view(torch.int16) if b.dtype == torch.bfloat16 else b), name
    if due:
        assert torch.equal(outs[1][3], outs[1][0])
        assert outs[1][5].abs().sum() > 0


def test_adam_matches_torch():
    n = 4099
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    step = torch.zeros(1, dtype=torch.int64, device=DEV)
    ref = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=1e-4, eps=1e-3)
    k = kernels()
    for _ in range(3):
        assert k.r2_adam(ptr(p), ptr(g), ptr(m), ptr(v), n, 1e-4, 0.9, 0.999, 1e-3, 1.0, ptr(step),
                         0, 0.0, stream_handle()) == 0
        step += 1
        ref.grad = g.clone()
        opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(p, ref.detach(), atol=1e-6, rtol=1e-5)


def test_sum_tree_sample_and_update():
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    cfg = get_config("reference", **{"replay.capacity": 70000, "replay.n_subrings": 7})
    rp = HBMReplay(cfg, DEV)
    rp.fill_synthetic(episode_len=120, seed=3)
    leaves = rp.tree[: rp.capacity].clone()
    total = rp.total_priority()
    assert abs(total - leaves.double().sum().item()) / total < 1e-4
    B = 4096
    idx = torch.zeros(B, dtype=torch.int32, device=DEV)
    prob = torch.zeros(B, device=DEV)
    rp.sample(B, idx, prob)
    torch.cuda.synchronize()
    il = idx.long()
    assert bool((leaves[il] > 0).all()), "sampled a row that is not a sequence start"
    assert torch.allclose(prob, leaves[il] / total, rtol=1e-4)
    # proportionality: chi-square-ish check on coarse bins
    bins = 14
    edges = torch.linspace(0, rp.capacity, bins + 1, device=DEV).long()
    exp = torch.stack([leaves[edges[i]:edges[i + 1]].sum() for i in range(bins)]) / total * B
    got = torch.histc(il.float(), bins=bins, min=0, max=rp.capacity)
    assert ((got - exp).abs() / exp.sqrt()).max() < 5.0
    # incremental update == full rebuild
    rp.priority[il[:100]] = 5.0
    rp.refresh_sequences(idx[:100], 100, 0, cfg.replay.seq_len)
    rp.update_tree()
    inc = rp.tree.clone()
    rp.rebuild_tree()
    torch.cuda.synchronize()
    assert torch.allclose(inc, rp.tree, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("cap", [1_000_000, 70_000])
def test_fused_tree_tail_matches_per_level_repair(cap):
    """replay.hip tree_update_tail_kernel: level-1 repair + upper levels by the last-arriving
    workgroup (+ step counter / dirty reset) == the per-level launches + step_end, bit for bit,
    three rounds in a row (the arrival ticket resets itself)."""
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    cfg = get_config("reference", **{"replay.capacity": cap, "replay.n_subrings": 8})
    a = HBMReplay(cfg, DEV)
    a.fill_synthetic(episode_len=120, seed=5)
    b = HBMReplay(cfg, DEV)
    b.fill_synthetic(episode_len=120, seed=5)
    assert a.tree_levels >= 4 and torch.equal(a.tree, b.tree)
    g = torch.Generator(device=DEV).manual_seed(cap)
    for rnd in range(3):
        B = 64
        idx = torch.zeros(B, dtype=torch.int32, device=DEV)
        prob = torch.zeros(B, device=DEV)
        a.sample(B, idx, prob)
        pr = torch.rand(cap, generator=g, device=DEV) * 3
        for r in (a, b):
            r.priority.copy_(pr)
            r.refresh_sequences(idx, B, 0, cfg.replay.seq_len)
        assert a.update_tree_and_end_step(True)
        b.update_tree()
        b.step_end()
        torch.cuda.synchronize()
        assert torch.equal(a.tree, b.tree), rnd
        assert int(a.step.item()) == int(b.step.item()) == rnd + 1
        assert int(a.dirty_count.item()) == 0 and int(a.tree_ticket.item()) == 0
    # without end_step the counter and the dirty list are left alone
    a.refresh_sequences(idx, 64, 0, cfg.replay.seq_len)
    n = int(a.dirty_count.item())
    assert a.update_tree_and_end_step(False)
    torch.cuda.synchronize()
    assert int(a.step.item()) == 3 and int(a.dirty_count.item()) == n


@pytest.mark.parametrize("cap", [1_000_000, 70_000])
def test_fused_prio_tail_matches_refresh_and_tree_repair(cap):
    """replay.hip prio_tail_kernel (sequence-priority refresh, grid barrier, level-0 repair, grid
    barrier, level-1 repair, last-arriver upper levels + step end, one launch) == refresh +
    the two-launch tree repair, bit for bit, rounds in a row (its counters reset themselves);
    windows of neighbouring samples overlap (shared leaves and parents across workgroups)."""
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    cfg = get_config("reference", **{"replay.capacity": cap, "replay.n_subrings": 8})
    a = HBMReplay(cfg, DEV)
    a.fill_synthetic(episode_len=120, seed=7)
    b = HBMReplay(cfg, DEV)
    b.fill_synthetic(episode_len=120, seed=7)
    assert torch.equal(a.tree, b.tree) and int(a.dirty_count.item()) == int(b.dirty_count.item())
    g = torch.Generator(device=DEV).manual_seed(cap + 1)
    for rnd in range(4):
        B = 64
        idx = torch.zeros(B, dtype=torch.int32, device=DEV)
        prob = torch.zeros(B, device=DEV)
        a.sample(B, idx, prob)
        if rnd == 3:
            idx[32:] = idx[:32]          # duplicate samples: identical windows in two workgroups
        pr = torch.rand(cap, generator=g, device=DEV) * 3
        for r in (a, b):
            r.priority.copy_(pr)
        assert a.prio_tail(idx, B, 0, cfg.replay.seq_len, end_step=True)
        b.refresh_sequences(idx, B, 0, cfg.replay.seq_len)
        assert b.update_tree_and_end_step(True)
        torch.cuda.synchronize()
        if not torch.equal(a.tree, b.tree):
            d = torch.nonzero(a.tree != b.tree).flatten().cpu()
            offs = [int(o) for o in a.tree_offs]
            lv = [sum(int(i) >= o for o in offs[1:]) for i in d[:8]]
            raise AssertionError(f"round {rnd}: {d.numel()} differ, first {d[:8].tolist()} levels {lv} "
                                 f"a {a.tree[d[:8]].tolist()} b {b.tree[d[:8]].tolist()} "
                                 f"offs {offs} sync {a.prio_sync.tolist()}")
        assert int(a.step.item()) == int(b.step.item()) == rnd + 1
        assert int(a.dirty_count.item()) == 0
        assert a.prio_sync.tolist() == [0] * 8, a.prio_sync.tolist()
    # without end_step the counter and the dirty list are left alone
    a.prio_tail(idx, 64, 0, cfg.replay.seq_len, end_step=False)
    torch.cuda.synchronize()
    assert int(a.step.item()) == 4 and int(a.dirty_count.item()) > 0


@pytest.mark.parametrize("skip", [0, 2])
def test_fused_prio_tail_sample_matches_tail_then_sample(skip):
    """replay.hip r2_prio_tail_sample (the hoisted step's side branch: priority tail ending the
    step, then the NEXT batch sampled from the repaired tree inside the same launch, the tail's
    workgroups kept off the first ``skip`` XCD slots) == prio_tail + sample_batch, bit for bit:
    tree, step counter, starts, probabilities, row list, stored states; the frame-queue words are
    zeroed; every sync word is back to 0."""
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    cfg = get_config("atari57", **{"replay.capacity": 64000, "replay.n_subrings": 8})
    a = HBMReplay(cfg, DEV)
    a.fill_synthetic(episode_len=200, seed=3)
    b = HBMReplay(cfg, DEV)
    b.fill_synthetic(episode_len=200, seed=3)
    B, H, Tn = 64, cfg.model.hidden, cfg.replay.seq_len + cfg.replay.n_step
    g = torch.Generator(device=DEV).manual_seed(9)
    z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=DEV)   # noqa: E731
    for rnd in range(3):
        idx = z(B, dt=torch.int32)
        a.sample(B, idx, z(B))
        pr = torch.rand(a.capacity, generator=g, device=DEV) * 3
        for r in (a, b):
            r.priority.copy_(pr)
        outs = []
        for r in (a, b):
            st, pb, rows = z(B, dt=torch.int32), z(B), z(Tn * B, dt=torch.int32)
            hs = [(r.hs_cs, 0, z(B, H), z(B, H)), (r.target_hs_cs, 5, z(B, H), z(B, H)),
                  (r.hs_cs, 5, z(B, H), z(B, H))]
            q = torch.full((4,), 7, dtype=torch.int32, device=DEV)
            outs.append((st, pb, rows, hs, q))
            if r is a:
                assert r.prio_tail_sample(idx, B, 40, 80, st, pb, rows, Tn, hs, True, q, skip_xcds=skip)
            else:
                assert r.prio_tail(idx, B, 40, 80, True)
                r.sample_batch(B, st, pb, rows, Tn, hs, h_f32=True, qreset=q)
        torch.cuda.synchronize()
        assert torch.equal(a.tree, b.tree) and torch.equal(a.step, b.step)
        (s0, p0, r0, h0, q0), (s1, p1, r1, h1, q1) = outs
        assert torch.equal(s0, s1) and torch.equal(p0, p1) and torch.equal(r0, r1)
        for (_, _, ha, ca), (_, _, hb, cb) in zip(h0, h1):
            assert torch.equal(ha, hb) and torch.equal(ca, cb)
        assert q0[:2].tolist() == [0, 0] and q0[2:].tolist() == [7, 7]
        assert a.prio_sync.tolist() == [0] * 8, a.prio_sync.tolist()
        assert int(a.dirty_count.item()) == 0


@pytest.mark.parametrize("N", [2560, 333])
def test_head_grads_and_colsum_match_torch(N):
    """gradsum.hip: dueling last-layer weight/bias grads, layer-1 bias grads and the permuted
    LSTM bias grads vs fp32 torch; bit-reproducible across launches (fixed-order reduction)."""
    k = kernels()
    g = torch.Generator(device=DEV).manual_seed(N)
    A, HD, G = 6, 256, 1024
    dva = torch.randn(N, 1 + A, generator=g, device=DEV)
    zr = torch.relu(torch.randn(N, 2 * HD, generator=g, device=DEV)).bfloat16()
    dz = torch.randn(N, 2 * HD, generator=g, device=DEV).bfloat16()
    dgates = torch.randn(N, G, generator=g, device=DEV).bfloat16()
    perm = torch.randperm(G, generator=torch.Generator().manual_seed(1)).to(DEV, torch.int32)
    ws = torch.zeros(int(k.r2_gradsum_ws_floats()), device=DEV)
    ticket = torch.zeros(64, dtype=torch.int32, device=DEV)
    outs = []
    for _ in range(2):
        gw2 = torch.full((1 + A, HD), float("nan"), device=DEV)
        gb2 = torch.full((1 + A,), float("nan"), device=DEV)
        gb1 = torch.full((2 * HD,), float("nan"), device=DEV)
        db = torch.full((G,), float("nan"), device=DEV)
        db2 = torch.full((G,), float("nan"), device=DEV)
        assert k.r2_head_grads(ptr(dva), ptr(zr), ptr(dz), ptr(gw2), ptr(gb2), ptr(gb1), N, A, HD,
                               ptr(ws), ptr(ticket), stream_handle()) == 0
        assert k.r2_colsum_bf16(ptr(dgates), N, G, ptr(perm), ptr(db), ptr(db2), ptr(ws),
                                ptr(ticket[32:]), stream_handle()) == 0
        torch.cuda.synchronize()
        outs.append((gw2, gb2, gb1, db, db2))
    gw2, gb2, gb1, db, db2 = outs[0]
    g2 = dva.t() @ zr.float()
    assert _rel(gw2[0], g2[0, :HD]) < 1e-5
    assert _rel(gw2[1:], g2[1:, HD:]) < 1e-5
    assert _rel(gb2, dva.sum(0)) < 1e-5
    assert _rel(gb1, dz.float().sum(0)) < 1e-5
    ref = torch.empty(G, device=DEV)
    ref[perm.long()] = dgates.float().sum(0)
    assert _rel(db, ref) < 1e-5 and torch.equal(db, db2)
    assert int(ticket.abs().sum().item()) == 0          # last arrivers reset their tickets
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("C,H,W,rows", [(3, 72, 96, True), (4, 84, 84, False), (3, 7, 5, True)])
def test_frames_gather_nhwc_matches_torch(C, H, W, rows):
    """torso.hip frames_gather_nhwc (vector form for HW % 4 == 0, scalar otherwise): replay
    uint8 (C,H,W) rows -> channels-last bf16, row list or identity, row stride > C*H*W."""
    from pytorch_r2d2_amd.ops.torso_lib import gather_frames_nhwc
    g = torch.Generator(device=DEV).manual_seed(C * H * W)
    frames = torch.randint(0, 256, (50, C * H * W + 16), dtype=torch.uint8, device=DEV, generator=g)
    idx = torch.randperm(50, device=DEV, generator=g)[:17].to(torch.int32) if rows else None
    x = gather_frames_nhwc(frames, idx, C, H, W)
    src = frames if idx is None else frames[idx.long()]
    ref = src[:, : C * H * W].view(-1, C, H, W).float()
    assert x.shape == ref.shape and x.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(x.float(), ref)
