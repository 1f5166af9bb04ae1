"""Library (MIOpen via ATen, channels-last bf16) conv-torso forward for frame geometries the fused
HIP torso kernels do not cover.  The fused kernels (csrc/kernels/torso.hip, torso_bwd.hip) are
specialised for the Atari torso: 4x84x84 uint8 stacks -> 32x20x20 -> 32x9x9 -> 32x7x7
(reference model.py:12-22); e.g. the DMLab-30 preset (3x72x96 RGB) runs here instead.
The outputs and saved activations use the same buffers/layouts as the fused path, so the rest of
the learner (LSTM, heads, TD, the library conv backward) is shared."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from ..config import EnvConfig, ModelConfig


def fused_torso_supported(env: EnvConfig, model: ModelConfig) -> bool:
    return (model.torso == "atari" and env.channels_per_frame * env.n_stacks == 4
            and env.frame_h == 84 and env.frame_w == 84 and tuple(model.conv_channels) == (32, 32, 32))


def torso_forward_library(frames: torch.Tensor, rows: Optional[torch.Tensor], layout, flat: torch.Tensor,
                          env: EnvConfig, model: ModelConfig, out: torch.Tensor,
                          act1: Optional[torch.Tensor] = None, act2: Optional[torch.Tensor] = None):
    """out (n, C3*h3*w3) bf16 = ReLU-conv stack of frames[rows] / 255 (frames stored (C,H,W) uint8
    per row); optionally saves conv1/conv2 activations channels-last into act1 / act2."""
    cin = env.channels_per_frame * env.n_stacks
    fh, fw = env.frame_h, env.frame_w
    x = frames if rows is None else frames.index_select(0, rows.long())
    n = x.shape[0]
    # uint8 0..255 is exact in bf16; the 1/255 of the reference's normalisation is folded into
    # the fp32 conv1 weights before their bf16 rounding (as the fused kernel applies it in fp32)
    x = x[:, : cin * fh * fw].view(n, cin, fh, fw).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    w = {k: layout.view(flat, k).to(torch.bfloat16) for k in
         ("vis_layers.0.bias", "vis_layers.2.weight", "vis_layers.2.bias",
          "vis_layers.4.weight", "vis_layers.4.bias")}
    w["vis_layers.0.weight"] = (layout.view(flat, "vis_layers.0.weight") * (1.0 / 255)).to(torch.bfloat16)
    y1 = F.conv2d(x, w["vis_layers.0.weight"], w["vis_layers.0.bias"], stride=4).relu_()
    y2 = F.conv2d(y1, w["vis_layers.2.weight"], w["vis_layers.2.bias"], stride=2).relu_()
    y3 = F.conv2d(y2, w["vis_layers.4.weight"], w["vis_layers.4.bias"], stride=1).relu_()
    out.copy_(y3.contiguous().view(n, -1))                   # torch (C,H,W) flatten order
    if act1 is not None:
        act1[:n].copy_(y1.permute(0, 2, 3, 1).reshape(n, -1, y1.shape[1]))
    if act2 is not None:
        act2[:n].copy_(y2.permute(0, 2, 3, 1).reshape(n, -1, y2.shape[1]))
