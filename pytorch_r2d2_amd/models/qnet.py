"""Recurrent dueling Q-network (R2D2 "QNet").

Parity target: ``/root/reference/model.py:6-83``.

* Conv torso ``Conv2d(4,32,8,s4)-ReLU-Conv2d(32,32,4,s2)-ReLU-Conv2d(32,32,3,s1)-ReLU``
  (``model.py:12-22``), flatten (C,H,W) order = 1568 features (``model.py:46``).
* ``LSTMCell(1568, 256)`` with PyTorch gate order (i, f, g, o) (``model.py:24``).
* Dueling head ``q = v + a - mean(a)`` (``model.py:26-36,62-64``).
* Stateful API: the recurrent state lives on the module between calls (``model.py:10,48-57``),
  ``reset/set_state/get_state`` (``model.py:76-83``).  ``forward`` accepts (T,B,C,H,W) or
  (B,C,H,W) and returns Q of shape (T*B, A) in time-major order (``model.py:38-74``).

The parameter names, shapes and ``state_dict`` keys are byte-compatible with the reference so
that ``save/{n}_save.pt`` checkpoints load in both directions.

This module is the *reference numerics* path (fp32 PyTorch ops, runs anywhere).  The MI355X
learner/actor hot paths do not call it: they run the hand-written HIP kernels in
``pytorch_r2d2_amd.ops`` on flat bf16 weight shadows (see ``engine.py``), and tests compare
those kernels against this module.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config import EnvConfig, ModelConfig


def conv_out(n: int, k: int, s: int) -> int:
    return (n - k) // s + 1


def torso_dims(env: EnvConfig, model: ModelConfig):
    """Return (in_channels, [(h,w) after each conv], flat_dim) for the conv torso."""
    cin = env.channels_per_frame * env.n_stacks
    h, w = env.frame_h, env.frame_w
    dims = []
    for k, s in ((8, 4), (4, 2), (3, 1)):
        h, w = conv_out(h, k, s), conv_out(w, k, s)
        dims.append((h, w))
    flat = model.conv_channels[2] * dims[-1][0] * dims[-1][1]
    return cin, dims, flat


class QNet(nn.Module):
    def __init__(self, device="cpu", model: Optional[ModelConfig] = None,
                 env: Optional[EnvConfig] = None, numpy_states: bool = True):
        super().__init__()
        self.model_cfg = model or ModelConfig()
        self.env_cfg = env or EnvConfig()
        self.device = device
        self.hs, self.cs = None, None
        # reference returns hs/cs as numpy (model.py:68-69); keep that for the compat API, the
        # engine never goes through this path.
        self.numpy_states = numpy_states
        m, e = self.model_cfg, self.env_cfg
        if m.torso == "atari":
            cin, _, flat = torso_dims(e, m)
            c1, c2, c3 = m.conv_channels
            self.in_shape = (cin, e.frame_h, e.frame_w)
            self.vis_layers = nn.Sequential(
                nn.Conv2d(cin, c1, kernel_size=8, stride=4), nn.ReLU(True),
                nn.Conv2d(c1, c2, kernel_size=4, stride=2), nn.ReLU(True),
                nn.Conv2d(c2, c3, kernel_size=3, stride=1), nn.ReLU(True),
            )
        elif m.torso == "mlp":
            self.in_shape = (e.obs_dim * e.n_stacks,)
            flat = m.mlp_hidden
            self.vis_layers = nn.Sequential(nn.Linear(self.in_shape[0], m.mlp_hidden), nn.ReLU(True))
        else:
            raise ValueError(m.torso)
        self.flat_dim = flat
        self.hidden = m.hidden
        self.n_actions = m.n_actions
        self.lstm = nn.LSTMCell(flat, m.hidden)
        self.val = nn.Sequential(nn.Linear(m.hidden, m.head_hidden), nn.ReLU(True),
                                 nn.Linear(m.head_hidden, 1))
        self.adv = nn.Sequential(nn.Linear(m.hidden, m.head_hidden), nn.ReLU(True),
                                 nn.Linear(m.head_hidden, m.n_actions))

    # ---- functional pieces (used by the reference learner and by kernel tests) ----
    def torso(self, x: torch.Tensor) -> torch.Tensor:
        """x: (N, *in_shape) float in [0,1] -> (N, flat)."""
        return self.vis_layers(x).reshape(x.shape[0], -1)

    def lstm_seq(self, xs: torch.Tensor, h: torch.Tensor, c: torch.Tensor):
        """xs: (T, B, D).  Returns h_seq (T,B,H), c_seq (T,B,H)."""
        hs, cs = [], []
        for t in range(xs.shape[0]):
            h, c = self.lstm(xs[t], (h, c))
            hs.append(h)
            cs.append(c)
        return torch.stack(hs), torch.stack(cs)

    def head(self, h: torch.Tensor) -> torch.Tensor:
        val = self.val(h)
        adv = self.adv(h)
        return val + adv - adv.mean(-1, keepdim=True)

    def seq_forward(self, state: torch.Tensor, h0: torch.Tensor, c0: torch.Tensor):
        """Stateless sequence forward.  state (T,B,*in_shape) -> q (T,B,A), h_seq, c_seq."""
        T, B = state.shape[:2]
        feats = self.torso(state.reshape(T * B, *state.shape[2:])).reshape(T, B, -1)
        h_seq, c_seq = self.lstm_seq(feats, h0, c0)
        return self.head(h_seq), h_seq, c_seq

    # ---- reference-compatible stateful API (model.py:38-83) ----
    def forward(self, state, return_hs_cs=False):
        n_in = len(self.in_shape)
        if state.dim() == n_in + 2:
            seq_size, batch_size = state.shape[:2]
        else:
            seq_size, batch_size = 1, state.shape[0]
        x = state.reshape(-1, *self.in_shape)
        feats = self.torso(x).reshape(seq_size, batch_size, -1)
        if self.hs is None:
            self.hs = torch.zeros(batch_size, self.hidden, device=feats.device)
            self.cs = torch.zeros(batch_size, self.hidden, device=feats.device)
        hs = torch.as_tensor(self.hs, dtype=feats.dtype, device=feats.device)
        cs = torch.as_tensor(self.cs, dtype=feats.dtype, device=feats.device)
        h_seq, c_seq = self.lstm_seq(feats, hs, cs)
        self.hs, self.cs = h_seq[-1], c_seq[-1]
        h_flat = h_seq.reshape(seq_size * batch_size, -1)
        c_flat = c_seq.reshape(seq_size * batch_size, -1)
        q_val = self.head(h_flat)
        if return_hs_cs:
            if self.numpy_states:
                return q_val, h_flat.detach().cpu().numpy(), c_flat.detach().cpu().numpy()
            return q_val, h_flat.detach(), c_flat.detach()
        return q_val

    def reset(self):
        self.hs, self.cs = None, None

    def set_state(self, hs, cs):
        self.hs, self.cs = hs, cs

    def get_state(self):
        return self.hs.detach().cpu().numpy(), self.cs.detach().cpu().numpy()


REFERENCE_STATE_DICT_SHAPES = {
    "vis_layers.0.weight": (32, 4, 8, 8), "vis_layers.0.bias": (32,),
    "vis_layers.2.weight": (32, 32, 4, 4), "vis_layers.2.bias": (32,),
    "vis_layers.4.weight": (32, 32, 3, 3), "vis_layers.4.bias": (32,),
    "lstm.weight_ih": (1024, 1568), "lstm.weight_hh": (1024, 256),
    "lstm.bias_ih": (1024,), "lstm.bias_hh": (1024,),
    "val.0.weight": (256, 256), "val.0.bias": (256,),
    "val.2.weight": (1, 256), "val.2.bias": (1,),
    "adv.0.weight": (256, 256), "adv.0.bias": (256,),
    "adv.2.weight": (6, 256), "adv.2.bias": (6,),
}


def value_rescale(x: torch.Tensor, eps: float = 1e-3) -> torch.Tensor:
    """h(x) = sign(x)(sqrt(|x|+1)-1) + eps*x  (R2D2 paper, absent in the reference)."""
    return torch.sign(x) * (torch.sqrt(x.abs() + 1.0) - 1.0) + eps * x


def value_rescale_inv(x: torch.Tensor, eps: float = 1e-3) -> torch.Tensor:
    """h^{-1}(x), closed form."""
    return torch.sign(x) * (((torch.sqrt(1.0 + 4.0 * eps * (x.abs() + 1.0 + eps)) - 1.0)
                             / (2.0 * eps)) ** 2 - 1.0)
