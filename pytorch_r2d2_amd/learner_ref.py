"""Pure-PyTorch R2D2 learner core (fp32, autograd).

Parity target: ``/root/reference/learner.py:68-104``.  This is the numerics oracle for the HIP
engine (tests compare the engine's loss / gradients / priorities against it) and the learner
used for configurations the HIP kernels do not cover (MLP torso / CartPole on CPU).

Sequence batch layout: ``frames`` (T+n, B, *obs) time-major, stored states at the sequence
start (and at +n for the reference/fixed modes), actions/rewards/dones of the learning rows.
The three ``target_mode`` variants are documented in ``engine/learner_engine.py``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import torch

from .config import R2D2Config
from .models.qnet import QNet, value_rescale, value_rescale_inv


@dataclass
class SeqBatch:
    obs: torch.Tensor          # (T+n, B, *obs) float
    h0: torch.Tensor           # (B, H) online stored state at s
    c0: torch.Tensor
    th0: torch.Tensor          # (B, H) target stored state (at s for shifted, s+n otherwise)
    tc0: torch.Tensor
    nh0: Optional[torch.Tensor]  # online stored state at s+n (fixed mode)
    nc0: Optional[torch.Tensor]
    action: torch.Tensor       # (Ll, B) long
    reward: torch.Tensor       # (Ll, B)
    done: torch.Tensor         # (Ll, B)
    weights: torch.Tensor      # (B,) IS weights (normalised); ones == reference


def _chain(net: QNet, obs, h, c, grad_from: int, grad_to: int):
    """Run net over obs (T,B,...) from (h,c); gradient flows only through steps
    [grad_from, grad_to) (burn-in and trailing steps are detached, learner.py:77-79)."""
    T, B = obs.shape[:2]
    qs = []
    feats_all = None
    with torch.no_grad():
        if grad_from > 0:
            f = net.torso(obs[:grad_from].reshape(grad_from * B, *obs.shape[2:])).reshape(grad_from, B, -1)
            hs, cs = net.lstm_seq(f, h, c)
            qs.append(net.head(hs))
            h, c = hs[-1], cs[-1]
    if grad_to > grad_from:
        n = grad_to - grad_from
        f = net.torso(obs[grad_from:grad_to].reshape(n * B, *obs.shape[2:])).reshape(n, B, -1)
        hs, cs = net.lstm_seq(f, h, c)
        qs.append(net.head(hs))
        h, c = hs[-1], cs[-1]
    if T > grad_to:
        with torch.no_grad():
            n = T - grad_to
            f = net.torso(obs[grad_to:].reshape(n * B, *obs.shape[2:])).reshape(n, B, -1)
            hs, cs = net.lstm_seq(f, h.detach(), c.detach())
            qs.append(net.head(hs))
    return torch.cat(qs, 0), (h, c)


def r2d2_loss(online: QNet, target: QNet, batch: SeqBatch, cfg: R2D2Config,
              mode: Optional[str] = None) -> Dict[str, torch.Tensor]:
    rc, lc = cfg.replay, cfg.learner
    mode = mode or lc.target_mode
    Lb, Ll, n = rc.burn_in, rc.learn, rc.n_step
    T = Lb + Ll
    obs = batch.obs
    if mode == "shifted":
        q_on, _ = _chain(online, obs, batch.h0, batch.c0, Lb, T)       # (T+n, B, A)
        with torch.no_grad():
            q_tg, _ = _chain(target, obs, batch.th0, batch.tc0, 0, 0)
        q_sa_all = q_on[Lb:T]
        q_arg = q_on[Lb + n:T + n].detach()
        q_tgt = q_tg[Lb + n:T + n]
    elif mode == "fixed":
        q_on, _ = _chain(online, obs[:T], batch.h0, batch.c0, Lb, T)
        with torch.no_grad():
            q_nx, _ = _chain(online, obs[n:], batch.nh0, batch.nc0, 0, 0)
            q_tg, _ = _chain(target, obs[n:], batch.th0, batch.tc0, 0, 0)
        q_sa_all = q_on[Lb:T]
        q_arg = q_nx[Lb:T]
        q_tgt = q_tg[Lb:T]
    elif mode == "reference":
        q_on, (h, c) = _chain(online, obs[:T], batch.h0, batch.c0, Lb, T)
        with torch.no_grad():
            q_nx, _ = _chain(online, obs[n + Lb:n + T], h.detach(), c.detach(), 0, 0)
            q_tg, _ = _chain(target, obs[n:], batch.th0, batch.tc0, 0, 0)
        q_sa_all = q_on[Lb:T]
        q_arg = q_nx
        q_tgt = q_tg[Lb:T]
    else:
        raise ValueError(mode)
    q_sa = q_sa_all.gather(2, batch.action.unsqueeze(-1)).squeeze(-1)          # (Ll, B)
    a_star = q_arg.argmax(-1, keepdim=True)
    boot = q_tgt.gather(2, a_star).squeeze(-1)
    if lc.value_rescale:
        boot = value_rescale_inv(boot, lc.value_rescale_eps)
    y = batch.reward + (lc.gamma ** n) * boot * (1.0 - batch.done)
    if lc.value_rescale:
        y = value_rescale(y, lc.value_rescale_eps)
    delta = q_sa - y.detach()
    loss = (batch.weights[None, :] * 0.5 * delta ** 2).mean()
    prio = (delta.detach().abs() + rc.priority_eps) ** rc.alpha
    return {"loss": loss, "delta": delta.detach(), "priority": prio, "q_sa": q_sa.detach(),
            "q_arg": q_arg.detach(), "q_tgt": q_tgt.detach()}


def batch_from_hbm(replay, starts: torch.Tensor, probs: Optional[torch.Tensor], cfg: R2D2Config,
                   device="cpu") -> SeqBatch:
    """Assemble a SeqBatch from an HBMReplay for given sequence starts (host-side, for tests)."""
    rc, H = cfg.replay, cfg.model.hidden
    Lb, Ll, n, T = rc.burn_in, rc.learn, rc.n_step, rc.seq_len
    s = starts.long().cpu()
    t = torch.arange(T + n)
    base = s - s % replay.cap_e
    rows = (base[None, :] + (s[None, :] - base[None, :] + t[:, None]) % replay.cap_e)  # (T+n, B)
    e = cfg.env
    if replay.obs is not None:
        obs = replay.obs[rows.to(replay.obs.device)].float()
    else:
        fr = replay.frames[rows.to(replay.frames.device)]
        obs = fr.view(T + n, len(s), e.channels_per_frame * e.n_stacks, e.frame_h, e.frame_w).float() / 255.0
    obs = obs.to(device)
    def st(buf, off):
        r = base + (s - base + off) % replay.cap_e
        v = buf[r.to(buf.device)].float().to(device)
        return v[:, :H].contiguous(), v[:, H:].contiguous()
    h0, c0 = st(replay.hs_cs, 0)
    toff = 0 if cfg.learner.target_mode == "shifted" else n
    th0, tc0 = st(replay.target_hs_cs, toff)
    nh0, nc0 = st(replay.hs_cs, n)
    lr = rows[Lb:T].to(replay.action.device)
    w = torch.ones(len(s), device=device)
    if probs is not None and rc.beta > 0:
        nv = max(int(replay.n_valid.item()), 1)
        w = (nv * probs.float().to(device).clamp_min(1e-30)) ** (-rc.beta)
        w = w / w.max()
    return SeqBatch(obs=obs, h0=h0, c0=c0, th0=th0, tc0=tc0, nh0=nh0, nc0=nc0,
                    action=replay.action[lr].long().to(device),
                    reward=replay.reward[lr].float().to(device),
                    done=replay.done[lr].float().to(device), weights=w)
