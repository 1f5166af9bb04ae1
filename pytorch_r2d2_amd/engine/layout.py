"""Flat parameter layout + packed bf16 kernel layouts.

All learnable parameters of one QNet live in ONE flat fp32 "master" buffer.  The same flat
layout is used for gradients, optimizer state and the data-parallel all-reduce buckets, so the
optimizer is a single launch (optim.hip) and the all-reduce moves two contiguous slices.

Segment order (chosen so that each backward GEMM writes its gradient straight into one
contiguous view):

    bucket "core" (LSTM + head; ~99% of the bytes, ready right after BPTT):
        lstm.weight_ih, lstm.weight_hh, lstm.bias_ih, lstm.bias_hh,
        val.0.weight, adv.0.weight      -> one (2*HD, H) view  (head hidden GEMM)
        val.0.bias, adv.0.bias          -> one (2*HD,) view
        val.2.weight, adv.2.weight      -> one (1+A, HD) view
        val.2.bias, adv.2.bias          -> one (1+A,) view
    bucket "torso" (conv weights; ready last):
        vis_layers.{0,2,4}.{weight,bias}

``state_dict()`` returns the reference key order and shapes (model.py:12-36), so checkpoints
are interchangeable with ``/root/reference``.

The kernels read bf16 copies in their own layouts, produced every optimizer step by ONE
``pack_bf16`` gather launch through a precomputed int32 index map:

    conv1  (C1, Cin*8*8)       k order (by, bx, ci, dy, dx), kh = 4by+dy, kw = 4bx+dx
                               (space-to-depth: 2x2 conv over a 21x21x64 image)
    conv2  (C2, 4*4*C1)        k order (kh, kw, ci)   channels-last implicit GEMM
    conv3  (C3, 3*3*C2)        k order (kh, kw, ci)
    w_ih   (G, D)  rows permuted to packed gate columns j*64 + g*16 + u  <- g*H + 16j + u
    w_hh   (NWG, 64, H)        same row permutation (recurrent GEMM B operand)
    w_hhT  (NWG, H, 64)        transposed slices (BPTT partial-dh GEMM B operand)
    head1  (2*HD, H)           [val.0.weight ; adv.0.weight]
and an fp32 gather for the small vectors: conv biases, packed LSTM biases, head vectors.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np
import torch

from ..config import EnvConfig, ModelConfig
from ..models.qnet import torso_dims

UNITS = 16  # hidden units per LSTM workgroup (csrc/kernels/lstm.hip LSTM_UNITS)


def gate_perm(H: int) -> np.ndarray:
    """perm[packed_col] = original gate row, packed = j*64 + g*16 + u, orig = g*H + 16j + u."""
    nwg = H // UNITS
    j, g, u = np.meshgrid(np.arange(nwg), np.arange(4), np.arange(UNITS), indexing="ij")
    return (g * H + UNITS * j + u).reshape(-1).astype(np.int64)


@dataclass
class Seg:
    name: str
    shape: Tuple[int, ...]
    offset: int

    @property
    def numel(self) -> int:
        return int(np.prod(self.shape))


class ParamLayout:
    def __init__(self, model: ModelConfig, env: EnvConfig):
        self.model, self.env = model, env
        H, HD, A = model.hidden, model.head_hidden, model.n_actions
        self.H, self.HD, self.A, self.G = H, HD, A, 4 * H
        if model.torso == "atari":
            cin, dims, flat = torso_dims(env, model)
            c1, c2, c3 = model.conv_channels
            torso = [("vis_layers.0.weight", (c1, cin, 8, 8)), ("vis_layers.0.bias", (c1,)),
                     ("vis_layers.2.weight", (c2, c1, 4, 4)), ("vis_layers.2.bias", (c2,)),
                     ("vis_layers.4.weight", (c3, c2, 3, 3)), ("vis_layers.4.bias", (c3,))]
            self.conv_dims = dims
            self.cin = cin
        else:
            flat = model.mlp_hidden
            obs = env.obs_dim * env.n_stacks
            torso = [("vis_layers.0.weight", (flat, obs)), ("vis_layers.0.bias", (flat,))]
            self.conv_dims = None
            self.cin = obs
        self.D = flat
        core = [("lstm.weight_ih", (4 * H, flat)), ("lstm.weight_hh", (4 * H, H)),
                ("lstm.bias_ih", (4 * H,)), ("lstm.bias_hh", (4 * H,)),
                ("val.0.weight", (HD, H)), ("adv.0.weight", (HD, H)),
                ("val.0.bias", (HD,)), ("adv.0.bias", (HD,)),
                ("val.2.weight", (1, HD)), ("adv.2.weight", (A, HD)),
                ("val.2.bias", (1,)), ("adv.2.bias", (A,))]
        self.segs: Dict[str, Seg] = OrderedDict()
        off = 0
        for name, shape in core:
            self.segs[name] = Seg(name, shape, off)
            off += int(np.prod(shape))
        self.core_numel = off
        off = (off + 3) // 4 * 4  # torso bucket starts 16-byte aligned
        self.torso_offset = off
        for name, shape in torso:
            self.segs[name] = Seg(name, shape, off)
            off += int(np.prod(shape))
        self.numel = off
        self.padded = (off + 3) // 4 * 4
        # module registration order of QNet == reference state_dict order (model.py:12-36)
        self.ref_order = [n for n, _ in torso] + [
            "lstm.weight_ih", "lstm.weight_hh", "lstm.bias_ih", "lstm.bias_hh",
            "val.0.weight", "val.0.bias", "val.2.weight", "val.2.bias",
            "adv.0.weight", "adv.0.bias", "adv.2.weight", "adv.2.bias"]
        self._build_pack_maps()

    # ------------------------------------------------------------------ views
    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        s = self.segs[name]
        return flat[s.offset:s.offset + s.numel].view(s.shape)

    def span(self, flat: torch.Tensor, first: str, last: str, shape) -> torch.Tensor:
        a, b = self.segs[first], self.segs[last]
        return flat[a.offset:b.offset + b.numel].view(shape)

    def views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {n: self.view(flat, n) for n in self.segs}

    def state_dict(self, flat: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
        return OrderedDict((n, self.view(flat, n).detach().cpu().clone()) for n in self.ref_order)

    def load_state_dict(self, flat: torch.Tensor, sd) -> None:
        for n in self.segs:
            if n not in sd:
                raise KeyError(f"missing key {n} in state_dict")
            v = self.view(flat, n)
            src = torch.as_tensor(sd[n])
            if tuple(src.shape) != tuple(v.shape):
                raise ValueError(f"shape mismatch for {n}: {tuple(src.shape)} vs {tuple(v.shape)}")
            v.copy_(src.to(v.device, v.dtype))

    def from_module(self, module, device) -> torch.Tensor:
        flat = torch.zeros(self.padded, dtype=torch.float32, device=device)
        self.load_state_dict(flat, module.state_dict())
        return flat

    # ------------------------------------------------------------------ packing
    def _build_pack_maps(self):
        """Index maps: packed_bf16[i] = master[bf_idx[i]], packed_f32[i] = master[f_idx[i]]."""
        H, HD, A, G, D = self.H, self.HD, self.A, self.G, self.D
        nwg = H // UNITS
        perm = gate_perm(H)
        off = lambda n: self.segs[n].offset  # noqa: E731
        bf: List[np.ndarray] = []
        self.bf_offsets: Dict[str, Tuple[int, Tuple[int, ...]]] = OrderedDict()
        cur = 0

        def add_bf(name, idx, shape):
            nonlocal cur
            idx = np.asarray(idx, dtype=np.int64).reshape(-1)
            self.bf_offsets[name] = (cur, tuple(shape))
            bf.append(idx)
            cur += idx.size
            pad = (-cur) % 8  # keep every packed tensor 16-byte aligned
            if pad:
                bf.append(np.full(pad, off("lstm.bias_ih"), dtype=np.int64))
                cur += pad

        if self.model.torso == "atari":
            c1, c2, c3 = self.model.conv_channels
            cin = self.cin
            # conv1 in space-to-depth order: the 8x8/s4 conv on (cin,84,84) is a 2x2/s1 conv on the
            # (21,21,16*cin) image with channel c = ci*16 + dy*4 + dx; k = (by*2+bx)*16cin + c
            co, by, bx, ci, dy, dx = np.meshgrid(np.arange(c1), np.arange(2), np.arange(2),
                                                 np.arange(cin), np.arange(4), np.arange(4),
                                                 indexing="ij")
            w1 = off("vis_layers.0.weight") + ((co * cin + ci) * 8 + 4 * by + dy) * 8 + 4 * bx + dx
            add_bf("conv1", w1, (c1, cin * 64))
            co, kh, kw, ci = np.meshgrid(np.arange(c2), np.arange(4), np.arange(4), np.arange(c1),
                                         indexing="ij")
            add_bf("conv2", off("vis_layers.2.weight") + ((co * c1 + ci) * 4 + kh) * 4 + kw,
                   (c2, 16 * c1))
            co, kh, kw, ci = np.meshgrid(np.arange(c3), np.arange(3), np.arange(3), np.arange(c2),
                                         indexing="ij")
            add_bf("conv3", off("vis_layers.4.weight") + ((co * c2 + ci) * 3 + kh) * 3 + kw,
                   (c3, 9 * c2))
            # backward (data-grad) layouts for the fused torso backward kernel:
            # conv3_dg[ci][kh][kw][co] = W3[co][ci][kh][kw]     (B[k=(kh,kw,co)][ci])
            ci, kh, kw, co = np.meshgrid(np.arange(c2), np.arange(3), np.arange(3), np.arange(c3),
                                         indexing="ij")
            add_bf("conv3_dg", off("vis_layers.4.weight") + ((co * c2 + ci) * 3 + kh) * 3 + kw,
                   (c2, 9 * c3))
            # conv2_dg[phase=(py,px)][ci][khi][kwi][co] = W2[co][ci][py+2khi][px+2kwi]
            py, px, ci, khi, kwi, co = np.meshgrid(np.arange(2), np.arange(2), np.arange(c1),
                                                   np.arange(2), np.arange(2), np.arange(c2),
                                                   indexing="ij")
            kh2, kw2 = py + 2 * khi, px + 2 * kwi
            add_bf("conv2_dg", off("vis_layers.2.weight") + ((co * c1 + ci) * 4 + kh2) * 4 + kw2,
                   (4, c1, 4 * c2))
        else:
            add_bf("mlp", off("vis_layers.0.weight") + np.arange(self.D * self.cin), (self.D, self.cin))
        permr = perm.reshape(nwg, 64)
        whhT = off("lstm.weight_hh") + permr[:, None, :] * H + np.arange(H)[None, :, None]
        add_bf("w_hhT", whhT, (nwg, H, 64))
        # W1^T (H, 2HD), k contiguous: B operand of the dh = dz @ W1 product fused into the TD
        # launch (td.hip r2_td_duel_dh)
        hh, kk = np.meshgrid(np.arange(H), np.arange(2 * HD), indexing="ij")
        add_bf("head1T", off("val.0.weight") + kk * H + hh, (H, 2 * HD))
        # the packs from here on are whole master rows in another row order (w_ih / w_hh: gate
        # permutation; head1: identity) -- the optimizer writes them itself (optim.hip
        # rmsprop_pack_kernel, one destination per master float4, rows are multiples of 4), the
        # pack launch only gathers the prefix above
        self.bf_rows_begin = cur
        add_bf("w_ih", off("lstm.weight_ih") + perm[:, None] * D + np.arange(D)[None, :], (G, D))
        add_bf("w_hh", off("lstm.weight_hh") + perm[:, None] * H + np.arange(H)[None, :],
               (nwg, 64, H))
        add_bf("head1", off("val.0.weight") + np.arange(2 * HD * H), (2 * HD, H))
        self.bf_numel = cur
        self.bf_index = torch.from_numpy(np.concatenate(bf).astype(np.int32))
        self.row_dst4 = self._row_dst4(np.concatenate(bf), self.bf_rows_begin)

        f: List[np.ndarray] = []
        self.f_offsets: Dict[str, Tuple[int, Tuple[int, ...]]] = OrderedDict()
        cur = 0

        def add_f(name, idx, shape):
            nonlocal cur
            idx = np.asarray(idx, dtype=np.int64).reshape(-1)
            self.f_offsets[name] = (cur, tuple(shape))
            f.append(idx)
            cur += idx.size
            pad = (-cur) % 4
            if pad:
                f.append(np.full(pad, off("lstm.bias_ih"), dtype=np.int64))
                cur += pad

        if self.model.torso == "atari":
            c1, c2, c3 = self.model.conv_channels
            add_f("b1", off("vis_layers.0.bias") + np.arange(c1), (c1,))
            add_f("b2", off("vis_layers.2.bias") + np.arange(c2), (c2,))
            add_f("b3", off("vis_layers.4.bias") + np.arange(c3), (c3,))
        else:
            add_f("mlp_b", off("vis_layers.0.bias") + np.arange(self.D), (self.D,))
        add_f("b_ih", off("lstm.bias_ih") + perm, (G,))
        add_f("b_hh", off("lstm.bias_hh") + perm, (G,))
        add_f("head_b1", off("val.0.bias") + np.arange(2 * HD), (2 * HD,))
        add_f("head_w2", off("val.2.weight") + np.arange((1 + A) * HD), (1 + A, HD))
        add_f("head_b2", off("val.2.bias") + np.arange(1 + A), (1 + A,))
        self.f_numel = cur
        self.f_index = torch.from_numpy(np.concatenate(f).astype(np.int32))
        # inverse gate permutation: orig col -> packed col (unpacking dgates for weight grads)
        inv = np.empty_like(perm)
        inv[perm] = np.arange(perm.size)
        self.gate_perm = torch.from_numpy(perm)
        self.gate_inv = torch.from_numpy(inv)

    def _row_dst4(self, idx: np.ndarray, begin: int):
        """(padded / 4) int32: the packed position of master float4 q when the packs at and after
        ``begin`` hold it as 4 consecutive elements at a 4-aligned position, else -1.  Every
        packed element from ``begin`` on (padding aside) must be covered exactly once, or None
        (the optimizer then does not write packs)."""
        dst = np.full(self.padded // 4, -1, dtype=np.int64)
        tail = idx[begin:].reshape(-1, 4)           # the packs are padded to 8 elements
        pad_v = self.segs["lstm.bias_ih"].offset
        run = (tail[:, 0] % 4 == 0) & np.all(np.diff(tail, axis=1) == 1, axis=1)
        q = tail[run, 0] // 4
        if np.unique(q).size != q.size:
            return None
        dst[q] = begin + 4 * np.nonzero(run)[0]
        if not np.all(run | np.all(tail == pad_v, axis=1)):
            return None
        return torch.from_numpy(dst.astype(np.int32))

    def torso_grad_map(self):
        """(dst index into the flat grad buffer, scale) for every element of the fused torso
        backward slab: [dW1 (co, ci*64) | dW2 (co, (kh,kw,ci)) | dW3 (co, (kh,kw,ci)) | db1 | db2 | db3]."""
        c1, c2, c3 = self.model.conv_channels
        off = lambda n: self.segs[n].offset  # noqa: E731
        cin = self.cin
        dst, scale = [], []
        dst.append(off("vis_layers.0.weight") + np.arange(c1 * cin * 64))
        scale.append(np.full(c1 * cin * 64, 1.0 / 255.0))
        co, kh, kw, ci = np.meshgrid(np.arange(c2), np.arange(4), np.arange(4), np.arange(c1), indexing="ij")
        dst.append((off("vis_layers.2.weight") + ((co * c1 + ci) * 4 + kh) * 4 + kw).reshape(-1))
        scale.append(np.ones(c2 * 16 * c1))
        co, kh, kw, ci = np.meshgrid(np.arange(c3), np.arange(3), np.arange(3), np.arange(c2), indexing="ij")
        dst.append((off("vis_layers.4.weight") + ((co * c2 + ci) * 3 + kh) * 3 + kw).reshape(-1))
        scale.append(np.ones(c3 * 9 * c2))
        for name, c in (("vis_layers.0.bias", c1), ("vis_layers.2.bias", c2), ("vis_layers.4.bias", c3)):
            dst.append(off(name) + np.arange(c))
            scale.append(np.ones(c))
        return (torch.from_numpy(np.concatenate(dst).astype(np.int32)),
                torch.from_numpy(np.concatenate(scale).astype(np.float32)))

    def packed_views(self, bf: torch.Tensor, f32: torch.Tensor):
        out = {}
        for n, (o, shp) in self.bf_offsets.items():
            out[n] = bf[o:o + int(np.prod(shp))].view(shp)
        for n, (o, shp) in self.f_offsets.items():
            out[n] = f32[o:o + int(np.prod(shp))].view(shp)
        return out

    def pack_torch(self, master: torch.Tensor, bf: torch.Tensor, f32: torch.Tensor) -> None:
        """Reference (pure torch) implementation of the pack kernels."""
        idx = self.bf_index.to(master.device).long()
        bf.copy_(master[idx].to(bf.dtype))
        fidx = self.f_index.to(master.device).long()
        f32.copy_(master[fidx])
