"""Loader for the in-tree gfx950 kernel library (``_r2d2_kernels.so``).

The library is loaded with ctypes *after* torch so that its ``libamdhip64.so.7`` dependency
binds to the HIP runtime torch already mapped.  On a machine with a GPU the library MUST be
present: ``kernels()`` raises instead of silently falling back to PyTorch, so a GPU run that
reports HIP numbers really ran the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch

_PKG = Path(__file__).resolve().parent.parent
_SO = _PKG / "_r2d2_kernels.so"
_lock = threading.Lock()
_lib = None

P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
F = ctypes.c_float

_SIGS = {
    "r2_abi_version": [],
    "r2_set_num_cus": [I],
    "r2_set_xcd_cus": [P],
    "r2_dp_local_stats": [P, P, P, I, P, P],
    "r2_dp_is_params": [P, I, I, F, P, P],
    "r2_get_num_cus": [],
    "r2_lstm_fwd": [P, I, I, I, I, I, P],
    "r2_lstm_bwd": [P, P, P, P, P, P, P, P, P, I, I, I, I, P],
    "r2_torso_fwd": [P, P, I, P, P, P, P, P, P, P, P, P, I, P],
    "r2_torso_fwd_multi": [P, P, I, I, I, I, P],
    "r2_torso_fwd_geom": [P, I64, P, I, I, I, I, I, I, I, P],
    "r2_frames_to_bf16": [P, P, I, P, P],
    "r2_frames_to_bf16_nhwc": [P, P, I, P, P],
    "r2_frames_gather_nhwc": [P, I64, P, I, I, I, F, P, P],
    "r2_bias_relu_nhwc_bf16": [P, P, I, I64, P],
    "r2_relu_mask_bf16": [P, P, P, I64, P],
    "r2_dueling_fwd": [P, P, P, P, P, P, I, I, I, P],
    "r2_dueling_bwd": [P, P, P, P, P, I, I, I, P],
    "r2_td_loss": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, I, F, F, F, F, P, P, P,
                   P],
    "r2_td_duel": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, I, F, F, F, F, P, P,
                   P, P, P, P, I, P, P, P],
    "r2_td_duel_dh": [P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, I, F, F, F, F, P, P,
                      P, P, P, P, I, P, P, P, P, P, I, P],
    "r2_dueling_fwd_multi_f32": [P, I, I, I, P],
    "r2_lstm_fwd_tag_sp": [P, I, I, I, I, P, P, P, P],
    "r2_lstm_bwd_tag_sp": [P, P, P, P, P, P, P, P, I, I, I, I, P, P, P, P, P, P, P, P],
    "r2_lstm_bwd_tag_sp_hg": [P, P, P, P, P, P, P, P, I, I, I, I, P, P, P, P, P, P, P,
                              P, P, P, P, P, P, P, I, I, I, P, P, P],
    "r2_tree_sample": [P, P, P, I, I, U64, P, P, P, P],
    "r2_tree_rebuild": [P, P, P, I, P],
    "r2_tree_update": [P, P, P, I, P, P, I, P],
    "r2_tree_update_fused": [P, P, P, I, P, P, I, P, P, P],
    "r2_tree_update_fused_reset": [P, P, P, I, P, P, I, P, P],
    "r2_seqprio_refresh": [P, I, P, P, P, I, I, I, I, F, P, P, I, P],
    "r2_mark_starts": [P, P, I, P, P, P, I, I, F, P, P, P, I, P],
    "r2_make_rows": [P, I, I, I, I, P, P],
    "r2_sample_batch": [P, P, P, I, I, U64, P, P, P, P, I, I, I, I, P, P, P, P, P],
    "r2_sample_batch_f32h": [P, P, P, I, I, U64, P, P, P, P, I, I, I, I, P, P, P, P, P],
    "r2_sample_batch_q": [P, P, P, I, I, U64, P, P, P, P, I, I, I, I, P, P, P, P, I, P, P],
    "r2_torso_fwd_sp_multi": [P, P, I, I, P],
    "r2_torso_sp_debug": [I],
    "r2_td_duel_set_done": [P],
    "r2_prio_tail_set_wait": [P],
    "r2_torso_sp_trace": [P],
    "r2_torso_bwd_sp_trace": [P],
    "r2_torso_bwd_sp_debug": [I],
    "r2_torso_bwd_sp": [P, P, I, P, P, P, P, P, P, P, P, P, P, P, P, I, P, P, P, P],
    "r2_torso_grad_reduce": [P, I, P, P, P, P],
    "r2_gather_state": [P, P, I, I, I, I, P, P, P, P],
    "r2_step_end": [P, P, P],
    "r2_rmsprop_centered": [P, P, P, P, I64, F, F, F, F, P, F, P],
    "r2_rmsprop_pack": [P, P, P, P, I64, F, F, F, F, P, F, P, P, P, I64, P, P, I64, P],
    "r2_rmsprop_pack_slab": [P, P, P, P, I64, F, F, F, F, P, P, P, I64, P, P, I64, P, I, I, P, P, I64, P],
    "r2_adam": [P, P, P, P, I64, F, F, F, F, F, P, P, F, P],
    "r2_sumsq": [P, I64, P, P],
    "r2_pack_bf16": [P, P, P, I64, P],
    "r2_gather_f32": [P, P, P, I64, P],
    "r2_copy_if_due": [P, P, I64, P, I64, P],
    "r2_noop_chain": [P, I, I, P],
    "r2_torso_bwd": [P, P, I, P, P, P, P, P, P, P, I, P, P, P, P],
    "r2_torso_bwd_slab_floats": [],
    "r2_torso_bwd_geom": [P, I64, P, I, P, P, P, P, P, P, P, I, P, P, P, I, I, I, P],
    "r2_torso_bwd_slab_floats_geom": [I, I, I],
    "r2_gemm": [P, I, P],
    "r2_gemm_set_version": [I],
    "r2_gemm_group": [P, P, I, P, I64, P, I, P],
    "r2_dueling_fwd_multi": [P, I, I, I, P],
    "r2_actor_pre": [P, P],
    "r2_actor_post": [P, P],
    "r2_actor_tail": [P, P],
    "r2_actor_args_bytes": [],
    "r2_pack_step": [P, P, I64, P, P, P, I64, P, P, P, I64, I64, I64, P, P, I64, P, I64, I64, P],
    "r2_pack_split": [P, P, P, I64, I64, P],
    "r2_torso_bwd_set_debug": [P],
    "r2_torso_fwd_set_debug": [P],
    "r2_lstm_persist_set_debug": [P],
    "r2_lstm_fwd_set_stamps": [P],
    "r2_td_duel_fwd_set": [P],
    "r2_prio_tail": [P, I, P, P, P, P, P, I, I, I, I, I, F, P, P, I, P, P, I, P],
    "r2_lstm_bwd_set_dz": [P, P, P, P, I],
    "r2_lstm_bwd_set_stop": [P, I, I],
    "r2_lstm_bwd_xcd_pairs": [I],
    "r2_lstm_probes": [],
    "r2_prio_tail_sample": [P, I, P, P, P, P, P, I, I, I, I, I, F, P, P, I, P, P, U64, P, P, P, I,
                            I, I, P, P, P, P, I, P, I, P],
    "r2_prio_tail_pack": [P, I, P, P, P, P, P, I, I, I, I, I, F, P, P, I, P, P, I,
                          P, P, I64, P, P, P, I64, P, P, P, I64, I64, I64, P, P, I64, I64, I64, P],
    "r2_td_duel_set_trace": [P],
    "r2_lstm_persist_force_slow": [I],
    "r2_xcc_probe": [P, I, I, I, P],
    "r2_gradsum_ws_floats": [],
    "r2_head_grads": [P, P, P, P, P, P, I, I, I, P, P, P],
    "r2_head_grads_sp": [P, P, P, P, P, P, P, I, I, I, P, P, P],
    "r2_colsum_bf16": [P, I, I, P, P, P, P, P, P],
    "r2_lstm_fwd_persist": [P, I, I, I, I, P, P, P],
    "r2_lstm_fwd_tag": [P, I, I, I, I, P, P, P, P],
    "r2_lstm_tag_ring_bytes": [I, I, I],
    "r2_lstm_bwd_tag": [P, P, P, P, P, P, I, I, I, I, P, P, P, P, P, P, P,
                        P, P, P, P, P, P, I, I, I, P, P, P],
    "r2_lstm_bwd_tag_hg_ok": [I, I, I],
    "r2_lstm_bwd_tag_ring_bytes": [I, I],
    "r2_lstm_bwd_persist": [P, P, P, P, P, P, P, I, I, I, I, P, P, P],
    "r2_apply_pending": [P, P, I, P, P, P, I, I, F, P, P, P, I, P, P],
    "r2_gemm5": [P, P, I, I, P, I64, P, I, I, P],
    "r2_gemm5_ws_bytes": [P, P, I, I],
    "r2_gemm5_ws_bytes_nc": [P, P, I, I, I],
    "r2_gemm5_set_mode": [I],
    "r2_ingest_record": [P, P],
    "r2_ingest_args_bytes": [],
    "r2_env_args_bytes": [],
    "r2_pack_args_bytes": [],
    "r2_pack_rows": [P, P],
    "r2_synth_env_step": [P, P],
    "r2_stream_create_cumask": [P, I, P],
    "r2_stream_get_cumask": [P, P, I],
    "r2_stream_destroy": [P],
    "r2_cu_probe": [P, I, I, P],
    "r2_memcpy_h2d_async": [P, P, I64, P],
    "r2_host_register": [P, I64],
    "r2_host_unregister": [P],
}


def library_path() -> Path:
    return _SO


def available() -> bool:
    return _SO.exists()


def kernels():
    """Return the loaded ctypes library, building it on first use if needed."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not _SO.exists():
            if os.environ.get("R2D2_NO_AUTOBUILD"):
                raise RuntimeError(f"{_SO} missing; run `python -m pytorch_r2d2_amd._build`")
            from .. import _build
            _build.build(verbose=False)
        torch.cuda.is_available()  # make sure torch's HIP runtime is mapped first
        lib = ctypes.CDLL(str(_SO), mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = argtypes
            fn.restype = ctypes.c_longlong if ("_ws_bytes" in name) else ctypes.c_int
        _lib = _Strict(lib)
        return _lib


class _Strict:
    """The loaded library with an argument-count check on every declared entry point: ctypes
    passes surplus arguments through as C varargs, so a stale call site (one argument list longer
    than the entry point's) would silently shift the trailing stream argument."""

    def __init__(self, lib):
        self._cdll = lib

    def __getattr__(self, name):
        fn = getattr(self._cdll, name)
        sig = _SIGS.get(name)
        if sig is None:
            return fn
        n = len(sig)

        def call(*args):
            if len(args) != n:
                raise TypeError(f"{name}: {len(args)} arguments, the entry point takes {n}")
            return fn(*args)

        call.__name__ = name
        self.__dict__[name] = call
        return call


def ptr(t) -> int:
    """Device/host pointer of a tensor (0 for None)."""
    if t is None:
        return 0
    return t.data_ptr()


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")
