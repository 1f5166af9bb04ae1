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
    """The whole fused torso (forward AND backward kernels): the Atari stack 4x84x84."""
    return (model.torso == "atari" and env.channels_per_frame * env.n_stacks == 4
            and env.frame_h == 84 and env.frame_w == 84 and tuple(model.conv_channels) == (32, 32, 32))


# frame geometries instantiated by the fused forward kernel (csrc/kernels/torso.hip TGeo)
FUSED_FWD_GEOMS = ((4, 84, 84), (3, 72, 96))


def fused_torso_fwd_geom(env: EnvConfig, model: ModelConfig):
    """(cin, h, w) when the fused bf16 torso FORWARD kernel covers this geometry (Atari 4x84x84,
    DMLab-30 RGB 3x72x96), else None."""
    g = (env.channels_per_frame * env.n_stacks, env.frame_h, env.frame_w)
    if model.torso == "atari" and tuple(model.conv_channels) == (32, 32, 32) and g in FUSED_FWD_GEOMS:
        return g
    return None


def torso_fwd_fused(frames: torch.Tensor, jobs, geom, grid: int, stream=None, reserve_xcds: int = 0,
                    reserve_slots: int = 0) -> None:
    """Launch the fused bf16 torso forward (torso.hip r2_torso_fwd_geom) over up to 4 frame-list
    jobs (rows of the uint8 replay / env frame buffer ``frames``; row stride from the tensor).
    ``jobs``: an (n, 12) int64 array kept alive by the caller (graph capture)."""
    from ._lib import check, kernels, ptr, stream_handle
    cin, h, w = geom
    check(kernels().r2_torso_fwd_geom(ptr(frames), frames.stride(0) * frames.element_size()
                                      if frames.dim() > 1 else cin * h * w,
                                      jobs.ctypes.data, len(jobs), grid, reserve_xcds, reserve_slots,
                                      cin, h, w, stream or stream_handle()), "torso_fwd_geom")


def gather_frames_nhwc(frames: torch.Tensor, rows: Optional[torch.Tensor], cin: int, fh: int,
                       fw: int, out: Optional[torch.Tensor] = None,
                       scale: float = 1.0) -> torch.Tensor:
    """(n, cin, fh, fw) bf16 view in channels-last memory of frames[rows] (uint8 (C,H,W) rows)
    * scale.  On the GPU one pass of torso.hip frames_gather_nhwc_kernel; on the CPU torch ops."""
    n = frames.shape[0] if rows is None else rows.numel()
    if frames.is_cuda:
        from ._lib import check, kernels, ptr, stream_handle
        if out is None:
            out = torch.empty((n, fh, fw, cin), dtype=torch.bfloat16, device=frames.device)
        r = None if rows is None else rows.to(torch.int32)
        check(kernels().r2_frames_gather_nhwc(ptr(frames), frames.stride(0), ptr(r), n, cin,
                                              fh * fw, float(scale), ptr(out), stream_handle()),
              "frames_gather_nhwc")
        return out.view(n, fh, fw, cin).permute(0, 3, 1, 2)
    x = frames if rows is None else frames.index_select(0, rows.long())
    x = (x[:, : cin * fh * fw].view(n, cin, fh, fw).float() * scale).to(torch.bfloat16)
    if out is not None:
        out.view(n, fh, fw, cin).copy_(x.permute(0, 2, 3, 1))
        return out.view(n, fh, fw, cin).permute(0, 3, 1, 2)
    return x.contiguous(memory_format=torch.channels_last)


def conv_relu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, stride: int) -> torch.Tensor:
    """ReLU(conv2d(x, w) + b): the MIOpen convolution without bias, then bias + ReLU in one
    in-place pass (torso.hip bias_relu_nhwc_kernel) on the channels-last output.  (MIOpen's own
    fused ``miopen_convolution_relu`` measured 24x slower here: 78 vs 3.3 ms per DMLab step.)"""
    y = F.conv2d(x, w, None, stride=stride)
    C = y.shape[1]
    if y.is_cuda and C % 8 == 0 and y.is_contiguous(memory_format=torch.channels_last):
        from ._lib import check, kernels, ptr, stream_handle
        bf = b.float().contiguous()
        check(kernels().r2_bias_relu_nhwc_bf16(ptr(y), ptr(bf), C, y.numel(), stream_handle()),
              "bias_relu_nhwc")
        return y
    return y.add_(b.view(1, -1, 1, 1)).relu_()


def torso_forward_library(frames: torch.Tensor, rows: Optional[torch.Tensor], layout, flat: torch.Tensor,
                          env: EnvConfig, model: ModelConfig, out: torch.Tensor,
                          act1: Optional[torch.Tensor] = None, act2: Optional[torch.Tensor] = None,
                          save_lo: int = 0):
    """out (n, C3*h3*w3) bf16 = ReLU-conv stack of frames[rows] / 255 (frames stored (C,H,W) uint8
    per row); optionally saves the conv1/conv2 activations of frames [save_lo, save_lo +
    len(act)) channels-last into act1 / act2."""
    cin = env.channels_per_frame * env.n_stacks
    fh, fw = env.frame_h, env.frame_w
    # uint8 0..255 is exact in bf16; the 1/255 of the reference's normalisation is folded into
    # the fp32 conv1 weights before their bf16 rounding (as the fused kernel applies it in fp32)
    x = gather_frames_nhwc(frames, rows, cin, fh, fw)
    n = x.shape[0]
    w = {k: layout.view(flat, k).to(torch.bfloat16) for k in
         ("vis_layers.0.bias", "vis_layers.2.weight", "vis_layers.2.bias",
          "vis_layers.4.weight", "vis_layers.4.bias")}
    w["vis_layers.0.weight"] = (layout.view(flat, "vis_layers.0.weight") * (1.0 / 255)).to(torch.bfloat16)
    y1 = conv_relu(x, w["vis_layers.0.weight"], w["vis_layers.0.bias"], 4)
    y2 = conv_relu(y1, w["vis_layers.2.weight"], w["vis_layers.2.bias"], 2)
    y3 = conv_relu(y2, w["vis_layers.4.weight"], w["vis_layers.4.bias"], 1)
    out.copy_(y3.contiguous().view(n, -1))                   # torch (C,H,W) flatten order
    for act, y in ((act1, y1), (act2, y2)):
        if act is not None:
            m = min(act.shape[0], n - save_lo)
            act[:m].copy_(y[save_lo:save_lo + m].permute(0, 2, 3, 1).reshape(m, -1, y.shape[1]))


def torso_forward_library_sp(frames: torch.Tensor, rows: Optional[torch.Tensor], layout,
                             flat: torch.Tensor, env: EnvConfig, model: ModelConfig,
                             out: torch.Tensor, out_lo: torch.Tensor,
                             act1: Optional[torch.Tensor] = None, act2: Optional[torch.Tensor] = None,
                             save_lo: int = 0):
    """fp32 (compute_dtype "fp32") library torso for geometries the split-precision fused kernel
    (torso_sp.hip, Atari 4x84x84 only) does not cover, e.g. DMLab-30 RGB 3x72x96: IEEE fp32 convs
    (MIOpen, NCHW), the features written as the (hi, lo) bf16 planes every split GEMM of
    the step reads (out + out_lo == the fp32 value to 2^-16 relative), the conv1 / conv2
    activations of frames [save_lo, ...) saved in fp32 for ``torso_backward_library_sp``."""
    cin = env.channels_per_frame * env.n_stacks
    # NCHW-contiguous fp32 throughout: MIOpen's most mature fp32 path (its NHWC fp32 backward
    # aborted the process on gfx950)
    x = gather_frames_nhwc(frames, rows, cin, env.frame_h, env.frame_w).float().contiguous()
    n = x.shape[0]
    v = lambda k: layout.view(flat, k)
    y1 = F.conv2d(x, v("vis_layers.0.weight") * (1.0 / 255), v("vis_layers.0.bias"), stride=4).relu_()
    y2 = F.conv2d(y1, v("vis_layers.2.weight"), v("vis_layers.2.bias"), stride=2).relu_()
    y3 = F.conv2d(y2, v("vis_layers.4.weight"), v("vis_layers.4.bias"), stride=1).relu_()
    y = y3.contiguous().view(n, -1)                            # torch (C,H,W) flatten order
    hi = y.to(torch.bfloat16)
    out.copy_(hi)
    out_lo.copy_(y - hi.float())
    for act, a in ((act1, y1), (act2, y2)):
        if act is not None:
            m = min(act.shape[0], n - save_lo)
            act[:m].copy_(a[save_lo:save_lo + m].permute(0, 2, 3, 1).reshape(m, -1, a.shape[1]))


def torso_backward_library_sp(frames: torch.Tensor, rows: torch.Tensor, layout, flat: torch.Tensor,
                              env: EnvConfig, model: ModelConfig, dims, dX: torch.Tensor,
                              dX_lo: torch.Tensor, X: torch.Tensor, act1: torch.Tensor,
                              act2: torch.Tensor, grad: torch.Tensor) -> None:
    """fp32 conv-torso backward of ``torso_forward_library_sp``: dX = hi + lo planes, ReLU masks
    from the saved activations (X: the forward's hi plane, > 0 exactly where the fp32 value is),
    IEEE fp32 ``convolution_backward``; the six torso gradients written into ``grad``."""
    cin = env.channels_per_frame * env.n_stacks
    c1, c2, c3 = model.conv_channels
    (h1, w1), (h2, w2), (h3, w3) = dims
    N = dX.shape[0]
    g3 = ((dX.float() + dX_lo.float()) * (X > 0)).view(N, c3, h3, w3)
    a2 = act2.view(N, h2, w2, c2).permute(0, 3, 1, 2).contiguous()
    a1 = act1.view(N, h1, w1, c1).permute(0, 3, 1, 2).contiguous()
    v = lambda k: layout.view(flat, k)
    cb = torch.ops.aten.convolution_backward
    d2, dw3, db3 = cb(g3, a2, v("vis_layers.4.weight"), [c3], [1, 1], [0, 0], [1, 1], False,
                      [0, 0], 1, [True, True, True])
    d1, dw2, db2 = cb(d2 * (a2 > 0), a1, v("vis_layers.2.weight"), [c2], [2, 2], [0, 0], [1, 1],
                      False, [0, 0], 1, [True, True, True])
    x = gather_frames_nhwc(frames, rows, cin, env.frame_h, env.frame_w).float().contiguous()
    _, dw1, db1 = cb(d1 * (a1 > 0), x, v("vis_layers.0.weight"), [c1], [4, 4], [0, 0], [1, 1],
                     False, [0, 0], 1, [False, True, True])
    for k, t in (("vis_layers.4.weight", dw3), ("vis_layers.4.bias", db3),
                 ("vis_layers.2.weight", dw2), ("vis_layers.2.bias", db2),
                 ("vis_layers.0.weight", dw1 * (1.0 / 255)), ("vis_layers.0.bias", db1)):
        layout.view(grad, k).copy_(t)
