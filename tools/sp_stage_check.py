"""Stage-by-stage error of the fp32 (split) engine forward vs float64 (debug aid)."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_split_gpu import _make, _oracle64, _rel  # noqa: E402
from pytorch_r2d2_amd.learner_ref import batch_from_hbm  # noqa: E402

cfg, rp, eng, net, tgt = _make("fixed", dtype=sys.argv[1] if len(sys.argv) > 1 else "fp32")
eng._forward_loss()
torch.cuda.synchronize()
on = net.double()
b = batch_from_hbm(rp, eng.starts, eng.probs, cfg, "cpu")
obs = b.obs.double()
Tn, B = obs.shape[:2]
with torch.no_grad():
    X = on.torso(obs.reshape(Tn * B, *obs.shape[2:]))
    Xe = eng.X_on.float().cpu().double() + (eng.X_on_lo.float().cpu().double() if eng.sp else 0)
    print("X      ", _rel(Xe, X))
    xp = X @ on.lstm.weight_ih.t() + on.lstm.bias_ih + on.lstm.bias_hh
    # engine xproj is in packed gate order: compare through the layout's permutation
    perm = eng.layout.gate_perm
    print("xproj  ", _rel(eng.xp_on.cpu().double(), xp[:, perm]))
    T = cfg.replay.seq_len
    hs, cs = on.lstm_seq(X.reshape(Tn, B, -1)[:T], b.h0.double(), b.c0.double())
    he = eng.hseq["on"].float().cpu().double() + (eng.hseq_lo["on"].float().cpu().double() if eng.sp else 0)
    print("h_seq  ", _rel(he, hs), " c_seq ", _rel(eng.cseq["on"].cpu().double(), cs))
    for t in (0, 3, T - 1):
        print(f"  h[{t}] ", _rel(he[t], hs[t]))
    Lb = cfg.replay.burn_in
    q = on.head(hs[Lb:]).reshape(-1, cfg.model.n_actions)
    print("q_on   ", _rel(eng.q_on.cpu().double(), q))
    print("h0 rel ", _rel(eng.h0["on"].float().cpu().double(), b.h0.double()))
