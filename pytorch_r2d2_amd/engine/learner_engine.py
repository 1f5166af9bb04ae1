"""MI355X learner engine: one R2D2 train step as a fixed sequence of HIP kernels.

Parity target: ``/root/reference/learner.py:68-120`` (train + interval).  The reference runs
5 QNet forward calls (each a Python loop of LSTMCell steps with a blocking D2H copy), a
36 MB H2D batch upload, autograd, torch.optim.RMSprop, a D2H of the TD errors and numpy
priority scatters.  Here a step is:

    sample    sample_batch: 64-ary sum-tree descent (device RNG keyed by the device step
              counter) -> time-major ring rows of the T+n frames -> stored (h, c) of every
              chain, one launch
    torso     fused uint8->conv1->conv2->conv3 MFMA kernel, every frame list of both nets in
              one multi-job launch
    proj      ONE MFMA GEMM launch for both nets: x . W_ih^T + (b_ih + b_hh), all T*B rows
    lstm      persistent recurrence kernel, all chains in one launch
    head      [val.0;adv.0] GEMM + fused dueling epilogue kernel (every head in one launch)
    td        fused double-Q n-step target / loss / dL/dQ / IS weights / row priorities, with
              the dueling head's backward (dz, dva) in the same launch (td_duel_kernel)
    backward  dh = dz W1 (on the TD launch's MFMAs), persistent BPTT (fused bias-gradient column sums;
              head-gradient reduction on its idle workgroups), weight-gradient + dX GEMMs in
              one grouped launch, fused conv backward from the saved activations
    allreduce (DP) bucket "core" beside the conv backward (which leaves CUs to RCCL), bucket
              "torso" beside the priority refresh + tree repair
    update    fused centered RMSprop (or Adam) over the flat master buffer, one pack launch
              producing every bf16 kernel layout, target sync as a device-side
              `copy_if_due` (graph-safe)
    priority  eta-mix refresh of every overlapping sequence + repair of every dirty sum-tree level
              + the step counter in ONE launch (replay.hip prio_tail_kernel, grid barriers between
              the levels; the 3-launch form when the grid cannot be resident)

No host synchronisation happens inside a step, so the whole step (minus collectives) is
captured once into a HIP graph and replayed.

target_mode (config.learner.target_mode):
  shifted   -- R2D2 paper: one online and one target chain over T+n frames from the stored
               state at the sequence start; Q(s_{t+n}) is read at offset +n (2 chains).
  fixed     -- the reference's 3-chain structure (online on state, target on next_state,
               online on next_state) with Q7 fixed: the online-on-next chain starts from the
               stored state at s+n and does its own burn-in.
  reference -- exactly learner.py:75-93 including Q7: online-on-next continues from the
               online-state chain's final state over next_state[burn_in:].
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import numpy as np
import torch

from ..config import R2D2Config
from ..models.qnet import QNet
from ..ops._lib import check, kernels, ptr, stream_handle
from ..ops.gemm import G5_CFGS, Gemm, gemm, gemm_group, gemm_sp, gemm_sp_ws_bytes, group_ws_bytes
from ..models.qnet import torso_dims
from ..ops.torso_lib import (fused_torso_fwd_geom, fused_torso_supported, gather_frames_nhwc,
                             torso_backward_library_sp, torso_forward_library,
                             torso_forward_library_sp, torso_fwd_fused)
from .layout import ParamLayout, UNITS
from .replay_hbm import HBMReplay


def _graph_upload(g) -> None:
    """Upload an instantiated graph's executable to the device (hipGraphUpload on the current
    stream), so its first replay -- possibly inside a timed loop -- does not pay for it.  Best
    effort: without the runtime entry point the first replay uploads as before."""
    import os
    try:
        exec_h = int(g.raw_cuda_graph_exec())
        lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        lib.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.hipGraphUpload(ctypes.c_void_p(exec_h), ctypes.c_void_p(stream_handle()))
    except (AttributeError, OSError, RuntimeError):
        pass


def _dispatch_serialized() -> bool:
    """True when kernel dispatches run one at a time (rocprofv3 counter collection / thread trace,
    AMD_SERIALIZE_KERNEL, HIP_LAUNCH_BLOCKING).  The hoisted step's early fork has a kernel on the
    side queue wait on the device for the TD kernel of the main queue, which a serialised
    dispatcher never runs beside it (a bounded stall and an error word), so it forks after TD there."""
    import os
    env = os.environ
    on = lambda k: env.get(k, "0").strip().lower() not in ("", "0", "false", "no", "off")  # noqa: E731
    return (on("ROCPROF_COUNTER_COLLECTION") or on("ROCPROF_ADVANCED_THREAD_TRACE")
            or on("HIP_LAUNCH_BLOCKING") or env.get("AMD_SERIALIZE_KERNEL", "0") not in ("", "0"))


def device_cus(device) -> int:
    """Multiprocessor (CU) count of ``device`` (256 on a whole MI355X; 256 for CPU tensors)."""
    d = torch.device(device)
    if d.type != "cuda":
        return 256
    return int(torch.cuda.get_device_properties(d).multi_processor_count)


def torso_bwd_grid(n_frames: int, reserve_cus: int = 0, n_cus: int = 256) -> int:
    """Workgroups of the fused conv backward (one per CU, grid-stride over frames).

    With ``reserve_cus`` > 0 (DP: the core gradient bucket's all-reduce runs beside it) the grid
    leaves at least that many CUs free, then shrinks further while the busiest workgroup's frame
    count stays the same: 2560 frames on 256 - 32 CUs is 12 frames per workgroup either way, so
    214 workgroups do it and 42 CUs go to RCCL at no extra conv time."""
    avail = max(8, n_cus - max(0, reserve_cus))
    if n_frames <= avail:
        return max(1, n_frames)
    if reserve_cus <= 0:
        return avail
    per = -(-n_frames // avail)
    return -(-n_frames // per)


class LearnerEngine:
    def _comm_reserve(self) -> int:
        dc = self.cfg.dist
        if self.dp and dc.overlap_allreduce and self.device.type == "cuda":
            return int(dc.comm_reserve_cus)
        return 0

    def __init__(self, cfg: R2D2Config, replay: HBMReplay, device="cuda", rank: int = 0,
                 world: int = 1, process_group=None, init_module: Optional[QNet] = None,
                 n_cus: Optional[int] = None, xcd_cus: Optional[List[int]] = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.replay = replay
        self.rank, self.world, self.pg = rank, world, process_group
        # data-parallel step machinery: world > 1, or forced at world 1 (dist.force_dp rehearsal)
        self.dp = bool(process_group is not None and (world > 1 or cfg.dist.force_dp))
        m, e, rc, lc = cfg.model, cfg.env, cfg.replay, cfg.learner
        if m.torso != "atari":
            raise NotImplementedError("the HIP engine runs the conv torso (Atari / DMLab frames); "
                                      "use the torch learner for vector observations")
        if m.hidden % UNITS != 0 or m.hidden not in (64, 128, 256, 512):
            raise NotImplementedError("LSTM kernels support hidden in {64,128,256,512}")
        self.layout = L = ParamLayout(m, e)
        d = self.device
        # compute units of THIS device (never assume 256: a partitioned MI355X exposes fewer); the
        # persistent kernels need their whole grid co-resident, one workgroup per CU.  ``n_cus``:
        # the CUs of the learner's CU-masked stream when it shares the chip (engine/concurrent.py)
        self.n_cus = int(n_cus) if n_cus else device_cus(d)
        if d.type == "cuda":
            kernels().r2_set_num_cus(self.n_cus)
            if xcd_cus is not None:     # a CU mask that is not an even split over the XCDs
                arr = (ctypes.c_int * 8)(*xcd_cus)
                kernels().r2_set_xcd_cus(arr)
            kernels().r2_lstm_persist_force_slow(0 if cfg.learner.lstm_xcd_pairs else 2)
        if init_module is None:
            torch.manual_seed(cfg.seed)
            init_module = QNet("cpu", m, e)
        self.master = L.from_module(init_module, d)
        if world > 1 and process_group is not None:
            # data-parallel ranks must start from identical weights: rank 0's are broadcast
            # (each rank seeds its own replay / env streams, never the model)
            import torch.distributed as dist
            src = dist.get_global_rank(process_group, 0) if hasattr(dist, "get_global_rank") else 0
            dist.broadcast(self.master, src=src, group=process_group)
        self.target = self.master.clone()
        self.grad = torch.zeros_like(self.master)
        self.opt_a = torch.zeros_like(self.master)
        self.opt_b = torch.zeros_like(self.master)
        self.bf_index = L.bf_index.to(d)
        self.row_dst4 = (L.row_dst4.to(d) if L.row_dst4 is not None and lc.fuse_opt_pack
                         else None)
        self.f_index = L.f_index.to(d)
        # split precision (compute_dtype "fp32", csrc/split.h): every bf16 kernel layout is packed as
        # a hi plane and a lo plane, (2, bf_numel); pk / pk_t view the hi planes, pk_lo / pk_t_lo
        # the lo planes
        self.sp = cfg.learner.compute_dtype == "fp32"
        if cfg.learner.compute_dtype not in ("fp32", "bf16"):
            raise ValueError(f"learner.compute_dtype must be fp32 or bf16, not {cfg.learner.compute_dtype!r}")
        nb = (2, L.bf_numel) if self.sp else (L.bf_numel,)
        self.bf = torch.zeros(nb, dtype=torch.bfloat16, device=d)
        self.f32 = torch.zeros(L.f_numel, dtype=torch.float32, device=d)
        self.bf_t = torch.zeros_like(self.bf)
        self.f32_t = torch.zeros_like(self.f32)
        self.lstm_b = torch.zeros(L.G, dtype=torch.float32, device=d)
        self.lstm_b_t = torch.zeros_like(self.lstm_b)
        if self.sp:
            self.pk = L.packed_views(self.bf[0], self.f32)
            self.pk_t = L.packed_views(self.bf_t[0], self.f32_t)
            self.pk_lo = L.packed_views(self.bf[1], self.f32)
            self.pk_t_lo = L.packed_views(self.bf_t[1], self.f32_t)
        else:
            self.pk = L.packed_views(self.bf, self.f32)
            self.pk_t = L.packed_views(self.bf_t, self.f32_t)
            self.pk_lo = self.pk_t_lo = None
        self.gate_inv = L.gate_inv.to(d)
        self.clip_buf = torch.zeros(1, dtype=torch.float32, device=d)
        self.steps_done = 0
        # data-parallel global prioritized sampling (parallel/sharded_replay.py)
        self.dp_global = bool(self.dp and cfg.dist.global_sampling)
        if self.dp_global and self.device.type == "cuda":
            # the 12-byte shard-stats all-gather runs on a side stream beside the torso / LSTM
            # graph segment.  It cannot starve the persistent forward: it depends on no kernel of
            # this step, so its RCCL workgroups finish once the peers reach the same collective;
            # and the forward's grid (one workgroup per CU, every member co-resident) must still
            # leave comm_reserve_cus CUs for them so the LSTM never waits for their exit
            chains = 2 if cfg.learner.target_mode == "shifted" else 3
            lstm_wgs = chains * -(-cfg.learner.batch_size // 16) * (cfg.model.hidden // UNITS)
            if lstm_wgs > self.n_cus - int(cfg.dist.comm_reserve_cus):
                raise ValueError(
                    f"DP global sampling: the persistent LSTM forward needs {lstm_wgs} co-resident "
                    f"workgroups, more than {self.n_cus} CUs minus dist.comm_reserve_cus="
                    f"{cfg.dist.comm_reserve_cus} left beside the shard-stats all-gather")
        self._duel_done = False       # the TD launch also ran the dueling-head backward
        self._dh_done = False         # ... and the dh = dz @ W1 product (learner.td_fuse_dh)
        self.graph = None
        self.stats: Dict[str, float] = {}
        self._alloc()
        if d.type == "cuda":
            # the BPTT packed two groups per XCD only beside the hoisted torso frames (alone it
            # runs faster one group per XCD: 100 vs 113 us, profiles/r06_hoist_bptt_placement.txt)
            kernels().r2_lstm_bwd_xcd_pairs(1 if self.hoist else 0)
        # world 1 (no gradient all-reduce, no clipping): the torso backward's slab reduction rides
        # on the optimizer launch (r2_rmsprop_pack_slab: one launch fewer); the torso bucket is the
        # master's tail, so the update's quad loop stops at its first quad
        self._fold_tq = None
        if (self.sp and not self.sp_lib and not self.dp and self.world == 1 and lc.fold_torso_reduce
                and lc.optimizer != "adam" and lc.grad_clip <= 0 and self.row_dst4 is not None
                and self.fwd_geom is not None and L.torso_offset % 4 == 0
                and bool((L.row_dst4[L.torso_offset // 4:] < 0).all())):
            self._fold_tq = L.torso_offset // 4
        self._pack(always=True)
        if d.type == "cuda":
            torch.cuda.synchronize(d)

    # ------------------------------------------------------------------ buffers
    def _alloc(self):
        cfg, d, L = self.cfg, self.device, self.layout
        rc, lc = cfg.replay, cfg.learner
        self.B = B = lc.batch_size
        self.Lb, self.Ll, self.n = rc.burn_in, rc.learn, rc.n_step
        self.T = T = rc.seq_len
        mode = lc.target_mode
        self.mode = mode
        H, D, G, A, HD = L.H, L.D, L.G, L.A, L.HD
        Lb, Ll, n = self.Lb, self.Ll, self.n
        self.Tn = Tn = T + n                      # frames per sequence touched
        self.Tc = Tn if mode == "shifted" else T  # chain length of the online chain
        bf16, f32 = torch.bfloat16, torch.float32
        z = lambda *s, dt=f32: torch.zeros(s, dtype=dt, device=d)  # noqa: E731
        sp = self.sp

        def zsp(*s):
            """An MFMA operand: bf16, or (split precision) a (2, *s) hi / lo pair -> (hi, lo)."""
            if sp:
                t = z(2, *s, dt=bf16)
                return t[0], t[1]
            return z(*s, dt=bf16), None
        # the MFMA operands an op reads as an fp32 value: fp32 in split precision, else bf16
        act_dt = f32 if sp else bf16
        self.starts = z(B, dt=torch.int32)
        self.probs = z(B)
        self.rows = z(Tn * B, dt=torch.int32)
        # hoisted target torso (learner.hoist): frame-queue words [side taken, next-step taken,
        # BPTT stop word, pad] (torso_sp.hip TSJob::q)
        self.tq = z(4, dt=torch.int32)
        self.X_on, self.X_on_lo = zsp(Tn * B, D)
        t_lo = 0 if mode == "shifted" else n       # first frame the target net needs
        self.t_lo_tg = t_lo
        self.X_tg, self.X_tg_lo = zsp((Tn - t_lo) * B, D)
        # conv activations of the learning frames, channels-last (N, h*w, c); the fused HIP torso
        # kernels cover the Atari geometry (4x84x84 -> 32x20x20 -> 32x9x9 -> 32x7x7), every other
        # geometry (e.g. DMLab RGB 3x72x96) runs the library conv path with the same buffers
        self.fused_torso = fused_torso_supported(cfg.env, cfg.model)
        # the fused FORWARD kernel also covers DMLab-30 RGB (3x72x96); its backward then runs on
        # the library convs from the saved activations
        self.fwd_geom = fused_torso_fwd_geom(cfg.env, cfg.model) if d.type == "cuda" else None
        if sp and not (cfg.model.torso == "atari" and d.type == "cuda" and L.H <= 256
                       and lc.lstm_impl == "persistent" and lc.lstm_handoff == "tagged"):
            raise NotImplementedError(
                "compute_dtype=fp32 (split precision) runs the conv torso, hidden <= 256 and the "
                "tagged persistent LSTM on a GPU; use compute_dtype=bf16 or the torch learner "
                "(learner_ref.py) for other configurations")
        # fp32 on a frame geometry the fused split torso (torso_sp.hip, Atari 4x84x84) does not
        # cover, e.g. DMLab-30 RGB: IEEE fp32 library convs feeding the same split planes
        self.sp_lib = sp and not self.fused_torso
        if self.sp_lib:
            torch.backends.cudnn.allow_tf32 = False     # the convs must stay IEEE fp32
        if (self.fwd_geom is None or lc.torso_bwd != "fused" or self.sp_lib) \
                and cfg.learner.conv_autotune and d.type == "cuda":
            # library conv path: let MIOpen benchmark its solutions once per shape (find mode);
            # DMLab-30: 463 -> 503 learner steps/s
            torch.backends.cudnn.benchmark = True
        if cfg.model.torso == "atari":
            cin, dims, _ = torso_dims(cfg.env, cfg.model)
            c1, c2, _c3 = cfg.model.conv_channels
            self.tdims = (cin, dims)
            if self.sp_lib:     # fp32 activations for the library backward
                self.act1, self.act1_lo = z(Ll * B, dims[0][0] * dims[0][1], c1), None
                self.act2, self.act2_lo = z(Ll * B, dims[1][0] * dims[1][1], c2), None
            else:
                self.act1, self.act1_lo = zsp(Ll * B, dims[0][0] * dims[0][1], c1)
                self.act2, self.act2_lo = zsp(Ll * B, dims[1][0] * dims[1][1], c2)
            self.frames_bf = z(Ll * B, cfg.env.frame_h * cfg.env.frame_w * cin, dt=bf16)
        self.h0 = {k: z(B, H, dt=act_dt) for k in ("on", "tg", "nx")}
        self.c0 = {k: z(B, H) for k in ("on", "tg", "nx")}
        self.hoist = self._hoist_ok()
        # the sampled batch (starts / probs / rows / stored states) in two sets: the hoisted step
        # k samples step k+1's batch into the other set while its own kernels still read set k % 2
        self._sets = [dict(starts=self.starts, probs=self.probs, rows=self.rows, h0=self.h0, c0=self.c0)]
        if self.hoist:
            self._sets.append(dict(starts=z(B, dt=torch.int32), probs=z(B), rows=z(Tn * B, dt=torch.int32),
                                   h0={k: z(B, H, dt=act_dt) for k in ("on", "tg", "nx")},
                                   c0={k: z(B, H) for k in ("on", "tg", "nx")}))
        self._cur = 0
        Tc = self.Tc
        self.hseq, self.hseq_lo = {}, {}
        self.hseq["on"], self.hseq_lo["on"] = zsp(Tc, B, H)
        self.hseq["tg"], self.hseq_lo["tg"] = zsp(T if mode != "shifted" else Tn, B, H)
        self.cseq = {"on": z(Tc, B, H), "tg": z(T if mode != "shifted" else Tn, B, H)}
        if mode != "shifted":
            Tnx = T if mode == "fixed" else Ll
            self.hseq["nx"], self.hseq_lo["nx"] = zsp(Tnx, B, H)
            self.cseq["nx"] = z(Tnx, B, H)
        self.gates = z(Tc - Lb, B, G)
        # head rows: online from Lb..Tc, target/next likewise
        self.Nh = (Tc - Lb) * B
        self.q_on = z(self.Nh, A)
        self.zr_on = z(self.Nh, 2 * HD, dt=act_dt)
        Ntg = (self.hseq["tg"].shape[0] - Lb) * B
        self.q_tg = z(Ntg, A)
        if mode != "shifted":
            Nnx = (self.hseq["nx"].shape[0] - (Lb if mode == "fixed" else 0)) * B
            self.q_nx = z(Nnx, A)
        self.dq = z(Ll * B, A)
        self.loss = z(1)
        self.td_abs = z(Ll * B)
        self.is_w = z(B)
        self.dz, self.dz_lo = zsp(Ll * B, 2 * HD)
        self.dva = z(Ll * B, 1 + A)
        nwg = H // UNITS
        self.slab0 = z(nwg, B, H)
        self.slab1 = z(nwg, B, H)
        self.dc = z(B, H)
        self.slab_p = z(2, nwg, B, H)
        self.ctr = z(int(kernels().r2_lstm_persist_ctr_words()), dt=torch.int32)
        # granule ring of the tagged forward hand-off (up to 4 chains per launch)
        self.ring = z(max(int(kernels().r2_lstm_tag_ring_bytes(4, B, H)), 16) // 4, dt=torch.int32)
        self.ring_b = z(max(int(kernels().r2_lstm_bwd_tag_ring_bytes(B, H)), 16) // 4, dt=torch.int32)
        self.bias_ws = z((B + 15) // 16, G)      # per-tile LSTM bias-gradient partials (tagged BPTT)
        self.err = z(1, dt=torch.int32)
        self.dgates, self.dgates_lo = zsp(Ll * B, G)
        self.gamma_n = float(lc.gamma ** n)
        self.td_part = z(4096)                          # TD loss partials, one per workgroup
        self.td_ticket = z(1, dt=torch.int32)           # reset by the kernel's last workgroup
        # the TD launch's done flag (hoisted step, early fork): set by its last workgroup, waited
        # on and cleared by the priority tail beside it
        self.td_done = z(1, dt=torch.int32) if self.device.type == "cuda" else None
        # fused torso backward: per-workgroup gradient slabs + destination map (allocated here,
        # never lazily: the step must be capturable without warm-up)
        if self.fwd_geom is not None:
            n_slab = int(kernels().r2_torso_bwd_slab_floats_geom(*self.fwd_geom))
            self._tb_grid = torso_bwd_grid(Ll * B, self._comm_reserve(), self.n_cus)
            self._tb_slab = z(self._tb_grid * n_slab)
            dst, scale = L.torso_grad_map()
            self._tb_dst, self._tb_scale = dst.to(d), scale.to(d)
        # every GEMM of the step is a hand-written MFMA kernel (gemm.hip / gemm_sp.hip): K and the
        # mn-major extents must be multiples of 8
        if not ((Ll * B) % 8 == 0 and D % 8 == 0 and H % 8 == 0 and (2 * HD) % 8 == 0 and G % 8 == 0):
            raise NotImplementedError(
                f"learn * batch ({Ll}*{B}), the torso width {D}, hidden {H} and head width {2 * HD} "
                "must be multiples of 8 (MFMA GEMM operands); use the torch learner (learner_ref.py)")
        self.use_gemm = True
        if A > 63 or HD % 64 != 0:
            raise NotImplementedError("the fused head kernels support <= 63 actions and a head "
                                      "width that is a multiple of 64")
        self.xp_on = z(Tn * B, G)
        self.xp_tg = z(self.X_tg.shape[0], G)
        self.z_on = z(self.Nh, 2 * HD, dt=act_dt)
        self.z_tg = z(Ntg, 2 * HD, dt=act_dt)
        if mode != "shifted":
            self.z_nx = z(Nnx, 2 * HD, dt=act_dt)
        self.dh = z(Ll * B, H)
        self.dX, self.dX_lo = zsp(Ll * B, D)
        self.gate_perm_i32 = L.gate_perm.to(d, torch.int32)
        self.gs_ws = torch.zeros(int(kernels().r2_gradsum_ws_floats()), dtype=torch.float32, device=d)
        self.gs_ticket = torch.zeros(64, dtype=torch.int32, device=d)
        # DP global sampling: local shard stats, the all-gathered (W, 3) stats, TD's 4 parameters
        self.dp_send = z(3)
        self.dp_recv = z(max(1, self.world) * 3)
        self.dp_params = z(4)

    # ------------------------------------------------------------------ weights
    def _pack(self, always: bool = False, stream=None):
        """Re-pack online weights (every step) and target weights (when synced)."""
        k = kernels()
        s = stream_handle(stream)
        L = self.layout
        if self.sp:
            check(k.r2_pack_split(ptr(self.master), ptr(self.bf_index), ptr(self.bf), L.bf_numel,
                                  L.bf_numel, s), "pack_split")
        else:
            check(k.r2_pack_bf16(ptr(self.master), ptr(self.bf_index), ptr(self.bf), L.bf_numel, s), "pack")
        check(k.r2_gather_f32(ptr(self.master), ptr(self.f_index), ptr(self.f32), L.f_numel, s), "gather")
        torch.add(self.pk["b_ih"], self.pk["b_hh"], out=self.lstm_b)
        if always:
            if self.sp:
                check(k.r2_pack_split(ptr(self.target), ptr(self.bf_index), ptr(self.bf_t), L.bf_numel,
                                      L.bf_numel, s), "pack_split_t")
            else:
                check(k.r2_pack_bf16(ptr(self.target), ptr(self.bf_index), ptr(self.bf_t), L.bf_numel, s),
                      "pack_t")
            check(k.r2_gather_f32(ptr(self.target), ptr(self.f_index), ptr(self.f32_t), L.f_numel, s), "gather_t")
            torch.add(self.pk_t["b_ih"], self.pk_t["b_hh"], out=self.lstm_b_t)

    def _pack_args(self, interval: int, rows_done: bool):
        """r2_pack_step's arguments from the master pointer to lo_off, the step counter excluded
        (the fused tail takes the counter from its own arguments)."""
        L = self.layout
        n_master, n_bf = (0, L.bf_rows_begin) if rows_done else (L.padded, L.bf_numel)
        return (ptr(self.master), ptr(self.target), n_master, ptr(self.bf_index), ptr(self.bf),
                ptr(self.bf_t), n_bf, ptr(self.f_index), ptr(self.f32), ptr(self.f32_t), L.f_numel,
                L.f_offsets["b_ih"][0], L.f_offsets["b_hh"][0], ptr(self.lstm_b), ptr(self.lstm_b_t),
                L.G), (interval, L.bf_numel if self.sp else 0)

    def _pack_step(self, interval: int, s, rows_done: bool = False):
        """rows_done: the optimizer already wrote the row packs and the target master
        (optim.hip rmsprop_pack_kernel): gather only the packs before layout.bf_rows_begin.
        With ``learner.fuse_pack_tail`` on the single-rank step the gather is deferred to the
        priority tail's launch instead (``_priorities``)."""
        if self._fuse_pack_tail() and rows_done:
            self._pack_deferred = (interval, rows_done)
            return
        head, tail = self._pack_args(interval, rows_done)
        check(kernels().r2_pack_step(*head, ptr(self.replay.step), *tail, s), "pack_step")

    def _fuse_pack_tail(self) -> bool:
        """The weight repack rides on the priority tail's launch (replay.hip r2_prio_tail_pack):
        single-rank step (the DP step runs the tail before the update), fused tail, GPU."""
        return (self.cfg.learner.fuse_pack_tail and not self.dp and self.device.type == "cuda"
                and self.cfg.replay.fused_prio_tail and not self.hoist)

    # ------------------------------------------------------------------ hoisted step
    # Single-rank split-precision step software-pipelined over two steps (round-6 verdict item
    # 1; reference: the serial /root/reference/learner.py:68-110).  Step k's priority tail needs
    # only its TD errors and step k+1's sample only the repaired tree, so right after the TD
    # launch a side stream runs [priority tail(k) + step counter, sample(k+1) into the other
    # sample set, target-net torso(k+1) frames from a queue] while the main stream runs the
    # BPTT and the rest of step k.  The side torso runs on the CUs the BPTT leaves free and stops
    # taking frames when the BPTT raises its stop word; step k+1's torso launch takes the rest of
    # the queue.  Every frame is computed by the same kernel code from the same operands, the
    # sample uses the same device step counter, and the target packs are only used when no
    # target sync happened in between (the host knows the sync steps: the update is captured with
    # the due decision baked in), so the step is bit-identical to the plain one.
    def _hoist_ok(self) -> bool:
        lc = self.cfg.learner
        return bool(lc.hoist and self.sp and self.fused_torso and not self.sp_lib
                    and self.device.type == "cuda" and not self.dp and lc.optimizer != "adam"
                    and self.row_dst4 is not None and self.cfg.replay.fused_prio_tail
                    and not lc.zero_stored_state and lc.grad_clip <= 0)

    def _use_set(self, i: int) -> None:
        self._cur = i
        S = self._sets[i]
        self.starts, self.probs, self.rows = S["starts"], S["probs"], S["rows"]
        self.h0, self.c0 = S["h0"], S["c0"]

    def invalidate_hoist(self) -> None:
        """Drop the batch the previous step sampled (and the target frames it computed) for the
        next one: call after changing the replay (ingest, actor writes) or the weights between
        steps.  The next step samples at its start, as the plain step does."""
        self._hoist_ready = False

    def _due(self, k: int) -> bool:
        iv = int(self.cfg.learner.target_update_interval)
        return iv <= 1 or (k + 1) % iv == 0

    def _baked_interval(self) -> int:
        """The target-sync interval handed to the update / pack kernels: the hoisted step's graph
        variants bake the due decision (1 = due, 2^62 = never), so the device step counter --
        already advanced by the side stream's priority tail -- is not read for it."""
        if not self.hoist:
            return int(self.cfg.learner.target_update_interval)
        return 1 if self._hoist_due else 1 << 62

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    def _hoist_side(self, torso: bool, after_td, td_wait: bool = False):
        """The side branch, forked at event ``after_td`` (recorded right after the TD launch):
        priority tail(k) + step counter, sample(k+1) into the other set (zeroing the frame
        queue), and (``torso``) the target-net frames of step k+1."""
        side = self._side_stream()
        side.wait_event(after_td)
        rp, B = self.replay, self.B
        nxt = 1 - self._cur
        with torch.cuda.stream(side):
            # one launch: the tail ends the step (counter + 1) and samples the next batch from the
            # repaired tree (replay.hip r2_prio_tail_sample); else the separate launches
            S, states = self._sample_dst(nxt)
            if td_wait:
                check(kernels().r2_prio_tail_set_wait(ptr(self.td_done)), "prio_tail_set_wait")
            ok = rp.prio_tail_sample(self.starts, B, self.Lb, self.T, S["starts"], S["probs"],
                                     S["rows"], self.Tn, states, self.sp, self.tq,
                                     skip_xcds=self._bptt_xcds())
            if not ok and td_wait:
                # refused on the host (shape / co-residency, e.g. ranks sharing the GPU): the
                # separate launches cannot wait for TD on the device, so this branch also waits for
                # the event after the TD launch; TD's unconsumed done flag is cleared, and this
                # engine stops forking early
                side.wait_event(self._early_post)
                self.td_done.zero_()
                self._early_refused = True
            if not ok:
                if not rp.prio_tail(self.starts, B, self.Lb, self.T, True):
                    rp.refresh_sequences(self.starts, B, self.Lb, self.T)
                    if not rp.update_tree_and_end_step(True):
                        rp.update_tree()
                        rp.step_end()
                self._sample(set_idx=nxt, qreset=self.tq)
            if torso:
                rows = self._sets[nxt]["rows"][self.t_lo_tg * B:]
                job = self._torso_job_sp(self.pk_t, self.pk_t_lo, rows, self.X_tg, self.X_tg_lo, qmode=1)
                arr = np.asarray([job], dtype=np.int64)
                self._side_job = arr      # (the launcher copies it into the kernel arguments)
                # every CU when the recurrence packs two groups per XCD (its helpers leave at
                # once), else the CUs outside its groups
                grid = (self.n_cus if self._bptt_pairs()
                        else max(1, self.n_cus - self._bptt_groups_wgs()))
                check(kernels().r2_torso_fwd_sp_multi(ptr(rp.frames), arr.ctypes.data, 1, grid,
                                                      stream_handle(side)), "torso_fwd_sp (hoisted)")
        return side

    def _bptt_pairs(self) -> bool:
        """The hoisted BPTT packs its recurrence groups two per XCD (lstm_persist.hip xcd_map 3,
        hidden / 16 = 16 workgroups a group; alone it runs faster one group per XCD, 97 vs 105
        us, so only beside the hoisted torso frames: profiles/r06_tree_ab_knobs.txt "np")."""
        return self.layout.H // UNITS == 16

    def _bptt_xcds(self) -> int:
        """The first n XCDs, which hold the BPTT recurrence's workgroups, for the hoisted
        branch's tail workgroups to stay off: ceil(batch tiles / 2) when packed in pairs."""
        return min(4, (-(-self.B // 16) + 1) // 2) if self._bptt_pairs() else 0

    def _bptt_groups_wgs(self) -> int:
        """Workgroups of the BPTT recurrence (batch tiles x hidden / 16)."""
        return -(-self.B // 16) * (self.layout.H // UNITS)

    def _hoist_body(self, p: int, inm: str, due: bool):
        """The hoisted step as stream operations (eager or captured): sample set ``p``; ``inm``
        'P' = sample at the start (no previous hoisted step), 'H' = the previous step sampled;
        ``due``: this step's update syncs the target (no target frames hoisted for the next
        step: they would use the old target weights)."""
        self._use_set(p)
        self._hoist_due = due
        if inm == "P":
            self._sample(qreset=self.tq)
        early = (bool(self.cfg.learner.hoist_early_fork) and self.td_done is not None
                 and not getattr(self, "_early_refused", False) and not _dispatch_serialized())
        if early:
            # fork before the TD launch (the side queue's start latency, ~13 us after its fork
            # event, then overlaps TD); the priority tail waits for TD's done flag on the device
            self._early_fork = torch.cuda.Event()
            self._early_post = None
        try:
            self._forward_rest()
        finally:
            after_td, self._early_fork = getattr(self, "_early_fork", None), None
        # (the fork is recorded only by the fused TD + head launch, td_fuse_head_bwd; without it
        # the side branch forks after TD as before)
        early = early and getattr(self, "_early_post", None) is not None
        main = torch.cuda.current_stream(self.device)
        if not early:
            after_td = torch.cuda.Event()
            after_td.record(main)
        # the BPTT and the weight-gradient group are issued (captured) BEFORE the side branch:
        # the graph keeps the first dependent of the TD node on the TD's queue, so the critical
        # path does not pay a cross-queue hand-off (measured: the BPTT started 11 us after the TD
        # when the side branch was captured first)
        self._backward_core()
        side = self._hoist_side(torso=not due, after_td=after_td, td_wait=early)
        # join before the conv backward: the side branch ends with the BPTT (joining at the end of
        # the step instead let the side torso slow the conv backward: measured slower)
        main.wait_stream(side)
        self._seg_torso()
        self._update()

    def _hoist_step(self):
        k = self.steps_done
        if getattr(self, "_dev_step_off", None) is None:
            self._dev_step_off = int(self.replay.step.item()) - k
        due = self._due(k + self._dev_step_off)
        p = k & 1
        inm = "H" if getattr(self, "_hoist_ready", False) else "P"
        if self.graph:
            self._use_set(p)
            self._hgraphs[(p, inm, due)].replay()
        else:
            self._hoist_body(p, inm, due)
        self._hoist_ready = True
        self.steps_done += 1

    def _chunk_len(self) -> int:
        return max(1, int(getattr(self.cfg.learner, "graph_chunk", 1))) if self.hoist else 1

    def run_steps(self, n: int) -> None:
        """``n`` learner steps, the same work and results as ``n`` calls of ``step``.  In the
        hoisted graph mode a run of ``learner.graph_chunk`` steps that starts at an even step,
        follows a hoisted step and has no target sync inside replays as ONE captured graph
        (the hoisted bodies back to back on the same streams): the ~5 us boundary between two
        graph replays (profiles/r06_step_timeline.txt) is paid once per chunk."""
        m = self._chunk_len()
        while n > 0:
            k = self.steps_done
            off = getattr(self, "_dev_step_off", None)
            if (n >= m and m > 1 and self.graph and getattr(self, "_cgraph", None) is not None
                    and (k & 1) == 0 and getattr(self, "_hoist_ready", False) and off is not None
                    and not any(self._due(k + j + off) for j in range(m))):
                self._use_set(0)
                self._cgraph.replay()
                self.chunks_run = getattr(self, "chunks_run", 0) + 1
                self._use_set((m - 1) & 1)
                self._hoist_due = False
                self.steps_done += m
                n -= m
            else:
                self.step()
                n -= 1

    def state_dict(self):
        return self.layout.state_dict(self.master)

    def target_state_dict(self):
        return self.layout.state_dict(self.target)

    def load_state_dict(self, sd, target_sd=None):
        self.layout.load_state_dict(self.master, sd)
        self.layout.load_state_dict(self.target, target_sd if target_sd is not None else sd)
        self._pack(always=True)
        self.invalidate_hoist()

    # ------------------------------------------------------------------ full state (resume)
    def full_state_extra(self) -> Dict[str, torch.Tensor]:
        """Optimizer moments + the device step counter (drives sampling RNG, Adam bias correction,
        target-sync cadence); with the weights this resumes a run exactly."""
        return {"opt_a": self.opt_a.detach().cpu().clone(), "opt_b": self.opt_b.detach().cpu().clone(),
                "replay_step": self.replay.step.detach().cpu().clone(),
                "steps_done": torch.tensor(self.steps_done)}

    def load_full_state(self, obj) -> None:
        """Restore from ``utils.checkpoint.load_full_checkpoint`` output (engine or Learner format)."""
        self.layout.load_state_dict(self.master, obj["online"])
        self.layout.load_state_dict(self.target, obj["target"])
        ex = obj.get("extra") or {}
        opt = obj.get("optimizer") or {}
        for name, buf in (("opt_a", self.opt_a), ("opt_b", self.opt_b)):
            v = ex.get(name, opt.get(name) if isinstance(opt, dict) else None)
            if v is not None:
                buf.copy_(v.to(buf.device))
        if "replay_step" in ex:
            self.replay.step.copy_(ex["replay_step"].to(self.replay.step.device))
        self.steps_done = int(ex["steps_done"]) if "steps_done" in ex else int(obj.get("step", 0))
        self._pack(always=True)
        self.invalidate_hoist()
        self._dev_step_off = None

    def sync_target(self):
        self.target.copy_(self.master)
        self._pack(always=True)
        self.invalidate_hoist()

    # ------------------------------------------------------------------ pieces
    def _chain_desc(self, xproj, pk, h0, c0, hseq, cseq, gates=None, save_from=0, pk_lo=None,
                    hseq_lo=None):
        d = [ptr(xproj), ptr(pk["w_hh"]), ptr(h0), ptr(c0), ptr(hseq), ptr(cseq), 0,
             ptr(gates), save_from]
        if self.sp:   # + W_hh lo plane, h_seq lo plane (h0 is fp32)
            d += [ptr(pk_lo["w_hh"]), ptr(hseq_lo)]
        return d

    def _lstm(self, chains, T, t_begin=0, site=0):
        k = kernels()
        arr = np.asarray([v for c in chains for v in c], dtype=np.int64)
        if self.sp:
            # the split-precision hand-off's 4-bit tags need one ring + ctr pair per launch site
            # (lstm_persist.hip lstm_fwd_tag_kernel T4): site 1 = the reference mode's nx chain
            if site == 0:
                ctr, ring = self.ctr, self.ring
            else:
                if not hasattr(self, "_site_bufs"):
                    z = lambda n: torch.zeros(n, dtype=torch.int32, device=self.device)
                    self._site_bufs = (z(int(k.r2_lstm_persist_ctr_words())),
                                       z(max(int(k.r2_lstm_tag_ring_bytes(4, self.B, self.layout.H)), 16) // 4))
                ctr, ring = self._site_bufs
            setattr(self, "_chain_arr%d" % site, arr)        # kept alive for capture
            check(k.r2_lstm_fwd_tag_sp(arr.ctypes.data, len(chains), self.B, T, self.layout.H,
                                       ptr(ctr), ptr(self.err), ptr(ring), stream_handle()),
                  "lstm_fwd_tag_sp")
            return
        if self.cfg.learner.lstm_impl == "persistent" and t_begin == 0:
            if self.cfg.learner.lstm_handoff == "tagged":
                rc = k.r2_lstm_fwd_tag(arr.ctypes.data, len(chains), self.B, T, self.layout.H,
                                       ptr(self.ctr), ptr(self.err), ptr(self.ring), stream_handle())
                if rc != -3:          # -3: grid too large for one workgroup per CU
                    check(rc, "lstm_fwd_tag")
                    return
            check(k.r2_lstm_fwd_persist(arr.ctypes.data, len(chains), self.B, T, self.layout.H,
                                        ptr(self.ctr), ptr(self.err), stream_handle()),
                  "lstm_fwd_persist")
        else:
            check(k.r2_lstm_fwd(arr.ctypes.data, len(chains), self.B, T, self.layout.H, t_begin,
                                stream_handle()), "lstm_fwd")

    def _heads(self, jobs, lo=None, duel: bool = True):
        """jobs: [(pk, h (N,H) bf16, z buffer, q out, zr out or None)].  Layer-1 GEMMs of all heads
        in one launch, then (``duel``) one dueling kernel for every head.  Split precision: ``lo`` =
        [(pk_lo, h lo plane)] per job; z / zr are fp32."""
        if self.sp:
            probs = [Gemm(h, pk["head1"].t(), zb, a_lo=hl, b_lo=pkl["head1"].t())
                     for (pk, h, zb, _, _), (pkl, hl) in zip(jobs, lo)]
            if self.cfg.learner.sp_gemm == "fused":
                # the launcher's CU model picks 128x128x64 (same-box sweep of the tile configs:
                # profiles/r03_heads_cfg_ab.txt)
                self._gemm_sp("heads", probs, splits=[0] * len(probs), cfg=-1)
            else:
                gemm(*probs)
            zs = [zb for _, _, zb, _, _ in jobs]
        else:
            gemm(*[Gemm(h, pk["head1"].t(), zb) for pk, h, zb, _, _ in jobs])
            zs = [zb for _, _, zb, _, _ in jobs]
        self._zs = zs
        if duel:
            self._duel_fwd(jobs, zs)

    def _duel_fwd(self, jobs, zs):
        # bias + ReLU + 512 -> 1+A + dueling combine of every head in one launch
        self._djobs = np.asarray([[ptr(z), ptr(pk["head_b1"]), ptr(pk["head_w2"]), ptr(pk["head_b2"]),
                                   ptr(q), ptr(zr), h.shape[0]]
                                  for (pk, h, _, q, zr), z in zip(jobs, zs)], dtype=np.int64)
        fn = kernels().r2_dueling_fwd_multi_f32 if self.sp else kernels().r2_dueling_fwd_multi
        check(fn(self._djobs.ctypes.data, len(jobs), self.layout.A, self.layout.HD, stream_handle()),
              "dueling_fwd")

    def _torso_job(self, pk, rows, out, save_at=None):
        B = self.B
        s1 = s2 = 0
        if save_at is not None:
            P1 = self.act1.shape[1] * self.act1.shape[2]
            P2 = self.act2.shape[1] * self.act2.shape[2]
            s1 = self.act1.data_ptr() + save_at * B * P1 * 2
            s2 = self.act2.data_ptr() + save_at * B * P2 * 2
        return [ptr(rows), rows.numel(), ptr(pk["conv1"]), ptr(pk["b1"]), ptr(pk["conv2"]),
                ptr(pk["b2"]), ptr(pk["conv3"]), ptr(pk["b3"]), ptr(out), s1, s2, 0]

    def _torso_job_sp(self, pk, pkl, rows, out, out_lo, save_at=None, qmode: int = 0):
        """torso_sp.hip job (20 int64): weights hi / lo, features hi / lo, saved activations, and
        (qmode 1 / 2, the hoisted step) the frame-queue words ``self.tq``."""
        B = self.B
        s = [0, 0, 0, 0]
        if save_at is not None:
            r0, r1 = save_at * B, save_at * B + rows.numel()
            s = [ptr(self.act1[r0:r1]), ptr(self.act1_lo[r0:r1]), ptr(self.act2[r0:r1]),
                 ptr(self.act2_lo[r0:r1])]
        q = [ptr(self.tq), qmode, 0] if qmode else [0, 0, 0]
        return [ptr(rows), rows.numel(), ptr(pk["conv1"]), ptr(pkl["conv1"]), ptr(pk["b1"]),
                ptr(pk["conv2"]), ptr(pkl["conv2"]), ptr(pk["b2"]), ptr(pk["conv3"]),
                ptr(pkl["conv3"]), ptr(pk["b3"]), ptr(out), ptr(out_lo)] + s + q

    # ------------------------------------------------------------------ the step
    def _forward_loss(self):
        self._sample()
        if self.dp_global:
            self._gather_dp()
        self._forward_rest()

    def _sample(self, set_idx: Optional[int] = None, qreset=None):
        """sample -> time-major row list -> stored recurrent states, one launch
        (replay_memory.py:224-262: multinomial over a host scan + per-row Python gathers).
        ``set_idx``: write that sample set (the hoisted step samples the next step's batch into
        the other set); ``qreset``: also zero the hoisted torso's frame-queue words."""
        B, Tn = self.B, self.Tn
        rp = self.replay
        if qreset is None and self.hoist:
            qreset = self.tq     # the torso launch after this sample takes every target frame
        S, states = self._sample_dst(self._cur if set_idx is None else set_idx)
        rp.sample_batch(B, S["starts"], S["probs"], S["rows"], Tn, states, h_f32=self.sp,
                        qreset=qreset)
        if self.cfg.learner.zero_stored_state:     # ablation: no stored recurrent state
            for _, _, h, c in states:
                h.zero_()
                c.zero_()
        if self.dp_global:
            root = rp.tree[int(rp.tree_offs[-1]): int(rp.tree_offs[-1]) + 1]
            if self.device.type == "cuda":     # one launch (dp_stats.hip)
                check(kernels().r2_dp_local_stats(ptr(root), ptr(rp.n_valid), ptr(self.probs), B,
                                                  ptr(self.dp_send), stream_handle()), "dp_local_stats")
            else:
                from ..parallel.sharded_replay import local_stats
                local_stats(root, rp.n_valid, self.probs, out=self.dp_send)

    def _sample_dst(self, i: int):
        """Sample set ``i`` and the stored-state gathers (hs_cs, row offset, h out, c out) of its
        chains."""
        rp, n = self.replay, self.n
        S = self._sets[i]
        h0, c0 = S["h0"], S["c0"]
        st_off = {"on": 0, "tg": 0 if self.mode == "shifted" else n, "nx": n}
        states = [(rp.hs_cs, 0, h0["on"], c0["on"]),
                  (rp.target_hs_cs, st_off["tg"], h0["tg"], c0["tg"])]
        if self.mode == "fixed":
            states.append((rp.hs_cs, n, h0["nx"], c0["nx"]))
        return S, states

    def _gather_dp(self):
        """The step's one extra collective (DP global sampling): 3 floats per rank."""
        from ..parallel.sharded_replay import gather_stats
        gather_stats(self.dp_send, self.world, self.pg, out=self.dp_recv, force=self.dp)

    def _forward_rest(self, tail: bool = True):
        """Torso, x-projections and recurrent chains; then (``tail``) heads, TD and priorities.
        DP global sampling needs the all-gathered shard stats only from the TD launch on, so the
        graphed DP step replays everything before ``_forward_tail`` while the 12-byte all-gather
        is in flight on its own stream (``step``)."""
        k = kernels()
        s = stream_handle()
        B, T, Tn, Lb, Ll, n = self.B, self.T, self.Tn, self.Lb, self.Ll, self.n
        L, rp, lc = self.layout, self.replay, self.cfg.learner
        H, A = L.H, L.A
        pk, pt = self.pk, self.pk_t
        rows = self.rows
        # torso: online over all Tn frames (save activations of the learning frames) and target
        if self.sp_lib:
            env, mc = self.cfg.env, self.cfg.model
            torso_forward_library_sp(rp.frames, rows, L, self.master, env, mc, self.X_on,
                                     self.X_on_lo, self.act1, self.act2, save_lo=Lb * B)
            torso_forward_library_sp(rp.frames, rows[self.t_lo_tg * B:], L, self.target, env, mc,
                                     self.X_tg, self.X_tg_lo)
        elif self.sp:
            pkl, ptl = self.pk_lo, self.pk_t_lo
            Xo, Xol, Xt, Xtl = self.X_on, self.X_on_lo, self.X_tg, self.X_tg_lo
            jobs = [self._torso_job_sp(pk, pkl, rows[: Lb * B], Xo[: Lb * B], Xol[: Lb * B]),
                    self._torso_job_sp(pk, pkl, rows[Lb * B: T * B], Xo[Lb * B: T * B],
                                       Xol[Lb * B: T * B], save_at=0),
                    self._torso_job_sp(pk, pkl, rows[T * B:], Xo[T * B:], Xol[T * B:]),
                    self._torso_job_sp(pt, ptl, rows[self.t_lo_tg * B:], Xt, Xtl,
                                       qmode=2 if self.hoist else 0)]
            jobs = [j for j in jobs if j[1] > 0]
            self._tjobs = np.asarray(jobs, dtype=np.int64)          # kept alive for capture
            check(k.r2_torso_fwd_sp_multi(ptr(rp.frames), self._tjobs.ctypes.data, len(jobs),
                                          self.n_cus, s), "torso_fwd_sp_multi")
        elif self.fwd_geom is not None:
            # one launch, workers dealt to the 4 jobs in proportion to their frames: separate
            # launches each ended in a partly idle last round of frames (18.6 us for the 320
            # tail frames alone)
            jobs = [self._torso_job(pk, rows[: Lb * B], self.X_on[: Lb * B]),
                    self._torso_job(pk, rows[Lb * B: T * B], self.X_on[Lb * B: T * B], save_at=0),
                    self._torso_job(pk, rows[T * B:], self.X_on[T * B:]),
                    self._torso_job(pt, rows[self.t_lo_tg * B:], self.X_tg)]
            jobs = [j for j in jobs if j[1] > 0]
            self._tjobs = np.asarray(jobs, dtype=np.int64)          # kept alive for capture
            torso_fwd_fused(rp.frames, self._tjobs, self.fwd_geom, self.n_cus, s)
        else:   # library convs: one call per net over all its frames (bigger, fewer launches)
            torso_forward_library(rp.frames, rows, L, self.master, self.cfg.env, self.cfg.model,
                                  self.X_on, self.act1, self.act2, save_lo=Lb * B)
            torso_forward_library(rp.frames, rows[self.t_lo_tg * B:], L, self.target, self.cfg.env,
                                  self.cfg.model, self.X_tg)
        # input projections (one GEMM per net over every row)
        if self.sp:
            xp_on, xp_tg = self.xp_on, self.xp_tg
            self._gemm_sp("xproj", [
                Gemm(self.X_on, pk["w_ih"].t(), xp_on, bias=self.lstm_b, a_lo=self.X_on_lo,
                     b_lo=self.pk_lo["w_ih"].t()),
                Gemm(self.X_tg, pt["w_ih"].t(), xp_tg, bias=self.lstm_b_t, a_lo=self.X_tg_lo,
                     b_lo=self.pk_t_lo["w_ih"].t())], splits=[0, 0])   # automatic K splits
        else:
            xp_on, xp_tg = self.xp_on, self.xp_tg
            gemm(Gemm(self.X_on, pk["w_ih"].t(), xp_on, bias=self.lstm_b),
                 Gemm(self.X_tg, pt["w_ih"].t(), xp_tg, bias=self.lstm_b_t))
        self._xp = (xp_on, xp_tg)
        G = L.G
        hl = self.hseq_lo
        pkl, ptl = self.pk_lo, self.pk_t_lo
        on = self._chain_desc(xp_on, pk, self.h0["on"], self.c0["on"], self.hseq["on"],
                              self.cseq["on"], self.gates, Lb, pkl, hl.get("on"))
        tg = self._chain_desc(xp_tg, pt, self.h0["tg"], self.c0["tg"], self.hseq["tg"], self.cseq["tg"],
                              None, 0, ptl, hl.get("tg"))
        if self.mode == "shifted":
            self._lstm([on, tg], self.Tc)
        elif self.mode == "fixed":
            nx = self._chain_desc(xp_on[n * B:], pk, self.h0["nx"], self.c0["nx"], self.hseq["nx"],
                                  self.cseq["nx"], None, 0, pkl, hl.get("nx"))
            self._lstm([on, tg, nx], T)
        else:  # reference: Q7 -- online-on-next continues from the online chain's final state
            self._lstm([on, tg], T)
            if self.sp:
                torch.add(self.hseq["on"][T - 1].float(), hl["on"][T - 1].float(), out=self.h0["nx"])
            else:
                self.h0["nx"].copy_(self.hseq["on"][T - 1])
            self.c0["nx"].copy_(self.cseq["on"][T - 1])
            nx = self._chain_desc(xp_on[(n + Lb) * B:], pk, self.h0["nx"], self.c0["nx"],
                                  self.hseq["nx"], self.cseq["nx"], None, 0, pkl, hl.get("nx"))
            self._lstm([nx], Ll, site=1)
        if tail:
            self._forward_tail()

    def _forward_tail(self):
        """Heads, TD loss and priorities (after every recurrent chain has run)."""
        k = kernels()
        s = stream_handle()
        B, Lb, Ll, n = self.B, self.Lb, self.Ll, self.n
        L, rp, lc = self.layout, self.replay, self.cfg.learner
        H, A = L.H, L.A
        pk, pt = self.pk, self.pk_t
        if self.dp_global:   # IS-weight parameters from the all-gathered shard stats
            if self.device.type == "cuda":     # one launch (dp_stats.hip)
                check(kernels().r2_dp_is_params(ptr(self.dp_recv), self.world, self.rank,
                                                float(self.cfg.replay.beta), ptr(self.dp_params),
                                                stream_handle()), "dp_is_params")
            else:
                from ..parallel.sharded_replay import global_is_params
                global_is_params(self.dp_recv.view(self.world, 3), self.rank,
                                 float(self.cfg.replay.beta), out=self.dp_params)
        # heads (rows from the first learning step on)
        jobs = [(pk, self.hseq["on"][Lb:].reshape(-1, H), self.z_on, self.q_on, self.zr_on),
                (pt, self.hseq["tg"][Lb:].reshape(-1, H), self.z_tg, self.q_tg, None)]
        lo = None
        if self.sp:
            hl = self.hseq_lo
            lo = [(self.pk_lo, hl["on"][Lb:].reshape(-1, H)), (self.pk_t_lo, hl["tg"][Lb:].reshape(-1, H))]
        if self.mode != "shifted":
            nx_from = Lb if self.mode == "fixed" else 0
            jobs.append((pk, self.hseq["nx"][nx_from:].reshape(-1, H), self.z_nx, self.q_nx, None))
            if self.sp:
                lo.append((self.pk_lo, self.hseq_lo["nx"][nx_from:].reshape(-1, H)))
        # fixed / reference modes: the three Q rows of transition i are row i of each head, so the
        # TD launch can run the dueling forward itself (td.hip td_duel_row)
        fuse_fwd = (lc.td_fuse_head_bwd and lc.td_fuse_head_fwd and self.mode != "shifted"
                    and A <= 32)
        self._heads(jobs, lo, duel=not fuse_fwd)
        if self.mode == "shifted":
            q_sa = self.q_on[: Ll * B]
            q_arg = self.q_on[n * B:(n + Ll) * B]
            q_tgt = self.q_tg[n * B:(n + Ll) * B]
        else:
            q_sa = self.q_on[: Ll * B]
            q_arg = self.q_nx[: Ll * B]
            q_tgt = self.q_tg[: Ll * B]
        rc = self.cfg.replay
        targs = (ptr(q_sa), ptr(q_arg), ptr(q_tgt), ptr(self.starts), ptr(self.probs),
                 ptr(rp.action), ptr(rp.reward), ptr(rp.done), ptr(self.dq), ptr(self.loss),
                 ptr(self.td_abs), ptr(rp.priority), ptr(self.is_w), ptr(rp.n_valid),
                 Ll, B, A, Lb, rp.cap_e, self.gamma_n, int(lc.value_rescale),
                 float(lc.value_rescale_eps), float(rc.alpha), float(rc.priority_eps),
                 float(rc.beta), ptr(self.td_part), ptr(self.td_ticket))
        dp = ptr(self.dp_params) if self.dp_global else 0
        # TD + the dueling head's backward in one launch (td.hip td_duel_kernel): dz / dva of the
        # online learning rows are written right where dL/dQ is known
        self._duel_done = False
        self._dh_done = False
        if lc.td_fuse_head_bwd:
            # + dh = dz @ W1 for the BPTT, on the same launch's MFMAs (16 rows per workgroup) --
            # unless the BPTT computes it itself (learner.bptt_dh, _dh_in_bptt)
            fuse_dh = lc.td_fuse_dh and L.H == 256 and not self._dh_in_bptt()
            w1t = ptr(pk["head1T"]) if fuse_dh else 0
            w1t_lo = ptr(self.pk_lo["head1T"]) if fuse_dh and self.sp else 0
            ef = getattr(self, "_early_fork", None)
            if ef is not None:
                # hoisted step, early fork: the side branch forks here, before the TD launch, and
                # its priority tail waits on the device for this launch's done flag
                ef.record(torch.cuda.current_stream(self.device))
                k.r2_td_duel_set_done(ptr(self.td_done))
            if fuse_fwd:
                z_on, z_tg, z_nx = self._zs[0], self._zs[1], self._zs[2]
                self._fwd_arr = np.asarray(
                    [ptr(z_on), ptr(z_nx), ptr(z_tg), ptr(pk["head_b1"]), ptr(pt["head_b1"]),
                     ptr(pt["head_w2"]), ptr(pk["head_b2"]), ptr(pt["head_b2"]), ptr(self.q_on),
                     ptr(self.q_nx), ptr(self.q_tg), 0], dtype=np.int64)
                k.r2_td_duel_fwd_set(self._fwd_arr.ctypes.data)
            rc_ = k.r2_td_duel_dh(*targs, ptr(self.zr_on[: Ll * B]), ptr(pk["head_w2"]), ptr(self.dz),
                                  ptr(self.dva), L.HD, ptr(self.dz_lo), dp, w1t, w1t_lo,
                                  ptr(self.dh) if fuse_dh else 0, L.H, s)
            if ef is not None and rc_ != 0:
                raise RuntimeError("td_duel refused the early-fork launch (code %d)" % rc_)
            if ef is not None:   # the fallback's fork point (_hoist_side: a refused fused tail)
                self._early_post = torch.cuda.Event()
                self._early_post.record(torch.cuda.current_stream(self.device))
            if rc_ == 0:
                self._duel_done = True
                self._dh_done = fuse_dh or self._dh_in_bptt()
                return
            if fuse_fwd:   # refused on the host before any launch: separate dueling forward
                k.r2_td_duel_fwd_set(None)
                self._duel_fwd(jobs, self._zs)
                fuse_fwd = False
            if self.sp:
                check(rc_, "td_duel")
        check(k.r2_td_loss(*targs, dp, s), "td_loss")

    def _dh_in_bptt(self) -> bool:
        """Split precision, hidden 256, head width 256: the BPTT computes its input gradient dh =
        dz . W1 itself (lstm_persist.hip PTBArgs::dz, 12 MFMAs per wave inside each hand-off wait)
        instead of the TD launch streaming all of W1^T through each of its workgroups."""
        lc, L = self.cfg.learner, self.layout
        return bool(self.sp and lc.bptt_dh and lc.td_fuse_head_bwd and L.H == 256 and 2 * L.HD == 512
                    and self.device.type == "cuda")

    def _backward_core_sp(self):
        """Split-precision backward core: head gradients, dh GEMM, BPTT, weight-gradient + dX
        GEMMs, every MFMA operand as hi / lo planes (the same launches as the bf16 path minus the
        BPTT side jobs)."""
        k = kernels()
        s = stream_handle()
        B, T, Lb, Ll = self.B, self.T, self.Lb, self.Ll
        L, pk, pkl = self.layout, self.pk, self.pk_lo
        H, A, HD, G = L.H, L.A, L.HD, L.G
        N = Ll * B
        g = self.grad
        gw2 = L.span(g, "val.2.weight", "adv.2.weight", (1 + A, HD))
        gb2 = L.span(g, "val.2.bias", "adv.2.bias", (1, 1 + A))
        gb1 = L.span(g, "val.0.bias", "adv.0.bias", (1, 2 * HD))
        hg = [ptr(self.dva), ptr(self.zr_on[:N]), ptr(self.dz), ptr(self.dz_lo), ptr(gw2), ptr(gb2),
              ptr(gb1), N, A, HD, ptr(self.gs_ws), ptr(self.gs_ticket)]
        # the head-gradient reduction rides on the BPTT launch's idle workgroups when they suffice
        # (as in the bf16 engine); otherwise it is its own launch
        side_hg = (self.cfg.learner.sp_head_grads_in_bptt and A <= 63
                   and bool(k.r2_lstm_bwd_tag_hg_ok(B, H, HD)))
        if not side_hg:
            check(k.r2_head_grads_sp(*hg, s), "head_grads_sp")
        dh = self.dh
        if not self._dh_done:   # else produced by the TD launch
            self._gemm_sp("dh", [Gemm(self.dz, pk["head1"], dh, a_lo=self.dz_lo, b_lo=pkl["head1"])],
                          splits=[0])
        bptt = [ptr(dh), ptr(self.gates), ptr(self.cseq["on"]), ptr(self.c0["on"]), ptr(pk["w_hhT"]),
                ptr(pkl["w_hhT"]), ptr(self.dgates), ptr(self.dgates_lo), B, T, Lb, H, ptr(self.ctr),
                ptr(self.err), ptr(self.ring_b), ptr(self.bias_ws), ptr(self.gate_perm_i32),
                ptr(L.view(g, "lstm.bias_ih")), ptr(L.view(g, "lstm.bias_hh"))]
        w_jobs, x_job = self._post_bptt_jobs()
        dz_on = self._dh_in_bptt() and self._duel_done
        if dz_on:
            check(k.r2_lstm_bwd_set_dz(ptr(self.dz), ptr(self.dz_lo), ptr(pk["head1T"]),
                                       ptr(pkl["head1T"]), 2 * HD), "lstm_bwd_set_dz")
        # the hoisted target torso beside this launch stops taking frames hoist_stop_lead
        # iterations before the recurrence ends; every helper takes head-gradient items
        lc = self.cfg.learner
        check(k.r2_lstm_bwd_set_stop(ptr(self.tq[2:]) if self.hoist else 0,
                                     max(0, self.Ll - int(lc.hoist_stop_lead)), 0),
              "lstm_bwd_set_stop")
        if side_hg:
            rc = k.r2_lstm_bwd_tag_sp_hg(*bptt, *hg, s)   # >= 0: bit 0 = head grads done here
        else:
            rc = k.r2_lstm_bwd_tag_sp(*bptt, s)
        check(min(rc, 0), "lstm_bwd_tag_sp")
        if side_hg and not rc & 1:
            check(k.r2_head_grads_sp(*hg, s), "head_grads_sp")
        self._dX = self.dX
        if self.cfg.learner.sp_gemm == "fused":
            probs = [w_jobs[2], w_jobs[1], w_jobs[0], x_job]
            sg, cfg = self.cfg.learner.sp_group_splits, self.cfg.learner.sp_group_cfg
            splits, auto_cfg = self._auto_group_splits(probs)
            if sg != "auto":
                splits = [int(v) for v in sg.replace(":", ",").split(",")][: len(probs)]
            self._gemm_sp("group", probs, splits, cfg=auto_cfg if cfg == -2 else cfg)
            return
        splits = self._group_splits(w_jobs, x_job)
        if splits:
            gemm_group([w_jobs[2], w_jobs[1], w_jobs[0], x_job], splits, self.gg_ws, self.gg_tickets)
        else:
            gemm(w_jobs[2], w_jobs[1], w_jobs[0])
            gemm(x_job)

    def _post_bptt_jobs(self):
        """The post-BPTT GEMMs of the split-precision step: [dW_head1, dW_hh, dW_ih], dX."""
        B, T, Lb, Ll = self.B, self.T, self.Lb, self.Ll
        L, pk, pkl = self.layout, self.pk, self.pk_lo
        H, HD = L.H, L.HD
        N = Ll * B
        g = self.grad
        hs, hl = self.hseq["on"], self.hseq_lo["on"]
        h_learn, h_learn_l = hs[Lb:T].reshape(N, H), hl[Lb:T].reshape(N, H)
        if Lb >= 1:
            h_prev, h_prev_l = hs[Lb - 1: T - 1].reshape(N, H), hl[Lb - 1: T - 1].reshape(N, H)
        else:   # the stored h0 (fp32) -> a split pair, then the chain's outputs
            if getattr(self, "_hprev_sp", None) is None:
                self._hprev_sp = torch.zeros(2, N, H, dtype=torch.bfloat16, device=self.device)
            h0 = self.h0["on"]
            hi0 = h0.to(torch.bfloat16)
            self._hprev_sp[0, :B].copy_(hi0)
            self._hprev_sp[1, :B].copy_((h0 - hi0.float()).to(torch.bfloat16))
            self._hprev_sp[0, B:].copy_(hs[: T - 1].reshape(-1, H))
            self._hprev_sp[1, B:].copy_(hl[: T - 1].reshape(-1, H))
            h_prev, h_prev_l = self._hprev_sp[0], self._hprev_sp[1]
        gw1 = L.span(g, "val.0.weight", "adv.0.weight", (2 * HD, H))
        X, Xl = self.X_on[Lb * B: T * B], self.X_on_lo[Lb * B: T * B]
        dgT, dgTl = self.dgates.t(), self.dgates_lo.t()
        w_jobs = [Gemm(self.dz.t(), h_learn, gw1, a_lo=self.dz_lo.t(), b_lo=h_learn_l),
                  Gemm(dgT, h_prev, L.view(g, "lstm.weight_hh"), crow=self.gate_perm_i32,
                       a_lo=dgTl, b_lo=h_prev_l),
                  Gemm(dgT, X, L.view(g, "lstm.weight_ih"), crow=self.gate_perm_i32, a_lo=dgTl, b_lo=Xl)]
        x_job = Gemm(self.dgates, pk["w_ih"], self.dX, a_lo=self.dgates_lo, b_lo=pkl["w_ih"],
                     c_lo=self.dX_lo)
        return w_jobs, x_job

    def _auto_group_splits(self, probs):
        """K splits of the post-BPTT group [dW_head1, dW_hh, dW_ih, dX] on 256 x 256 tiles: the
        weight gradients (K = learn x batch) split 4 ways when they have >= 32 K steps (paper
        config: 80), else 1 (a split's partial-tile write + reduction outweighs 1-3 K steps);
        dX (K = 4H) takes the largest of 4 / 2 ways whose items still fit one round on the CUs.
        Measured: paper 4,4,4,1 (profiles/r04_group_splits_ab.txt: 3,4,4,2 / 3,5,5,2 slower);
        reference config 1,1,1,4 = 0.2455 ms vs 0.3038 at 4,4,4,1.
        Returns (splits, tile config for learner.sp_group_cfg = -2).  Round 5
        (tools/wgrad_probe.py, profiles/r05_wgrad_group_ab.txt): at >= 32 dW K steps the 128x128
        tile with a 4-deep 32-K ring (G5_CFGS[6]) and splits 3,3,3,1 runs the paper group in
        97 us vs 113 on 256x256 tiles at 4,4,4,1 (same-box step -1.6 %): the 384 + 260 smaller
        items balance over the CUs and each split's last-arriver reduction reads 3 x 64 KB, not
        4 x 256 KB."""
        t = lambda g: -(-g.a.shape[0] // 256) * -(-g.b.shape[1] // 256)   # noqa: E731
        ks_w = -(-probs[0].a.shape[1] // 32)
        if ks_w >= 32:
            return [3, 3, 3, 1], 6
        sw = 1
        items = sw * sum(t(g) for g in probs[:3])
        sx = next((c for c in (4, 2) if items + c * t(probs[3]) <= self.n_cus), 1)
        return [sw, sw, sw, sx], -1

    def _gemm_sp(self, site: str, probs, splits=None, cfg: int = -1):
        """Split-precision GEMMs of one call site: the fused one-pass kernel (gemm_sp.hip) with a
        per-site split-K workspace sized before capture, or the multi-pass kernels
        (``learner.sp_gemm``)."""
        if self.cfg.learner.sp_gemm != "fused":
            gemm(*probs)
            return
        splits = splits or [1] * len(probs)
        if not hasattr(self, "_sp_ws"):
            self._sp_ws = {}
        cur = self._sp_ws.get(site)
        if cur is None:   # (inside a capture: from the graph's pool, kept alive here)
            need = max(gemm_sp_ws_bytes(probs, splits, c, self.n_cus) for c in range(len(G5_CFGS)))
            cur = (torch.zeros(max(need // 4, 1), dtype=torch.float32, device=self.device),
                   torch.zeros(4096, dtype=torch.int32, device=self.device))
            self._sp_ws[site] = cur
        gemm_sp(probs, splits=splits, cfg=cfg, ws=cur[0], tickets=cur[1], n_cus=self.n_cus)

    def _backward_core(self):
        """Head backward, BPTT, LSTM/head weight gradients -> grad bucket 'core'."""
        if self.sp:
            return self._backward_core_sp()
        k = kernels()
        s = stream_handle()
        B, T, Lb, Ll = self.B, self.T, self.Lb, self.Ll
        L, pk = self.layout, self.pk
        H, A, HD, G = L.H, L.A, L.HD, L.G
        N = Ll * B
        zr = self.zr_on[:N]
        if not self._duel_done:      # else fused into the TD launch
            check(k.r2_dueling_bwd(ptr(self.dq), ptr(zr), ptr(pk["head_w2"]), ptr(self.dz),
                                   ptr(self.dva), N, A, HD, s), "dueling_bwd")
        g = self.grad
        gw2 = L.span(g, "val.2.weight", "adv.2.weight", (1 + A, HD))
        gb2 = L.span(g, "val.2.bias", "adv.2.bias", (1, 1 + A))
        gb1 = L.span(g, "val.0.bias", "adv.0.bias", (1, 2 * HD))
        # gradsum.hip head_grads (any head up to 63 actions: Seaquest 18, DMLab 15): last-layer
        # weight / bias grads and the layer-1 bias grads in one deterministic column reduction,
        # on the tagged BPTT launch's idle workgroups when they are enough, else its own launch
        self._hg_job = [ptr(self.dva), ptr(zr), ptr(self.dz), ptr(gw2), ptr(gb2), ptr(gb1),
                        N, A, HD, ptr(self.gs_ws), ptr(self.gs_ticket)]
        h_learn = self.hseq["on"][Lb:T].reshape(N, H)
        gw1 = L.span(g, "val.0.weight", "adv.0.weight", (2 * HD, H))
        dh = self.dh
        if not self._dh_done:        # else dh = dz W1 ran on the TD launch's MFMAs
            gemm(Gemm(self.dz, pk["head1"], dh))
        X = self.X_on[Lb * B: T * B]
        if Lb >= 1:
            h_prev = self.hseq["on"][Lb - 1: T - 1].reshape(N, H)
        else:
            h_prev = torch.cat([self.h0["on"][None], self.hseq["on"][: T - 1]]).reshape(N, H)
        # weight gradients straight into the flat buffer; the row map puts the packed gate order
        # back into torch order (no gather of dgates, no copies)
        dgT = self.dgates.t()
        w_jobs = [Gemm(self.dz.t(), h_learn, gw1),
                  Gemm(dgT, h_prev, L.view(g, "lstm.weight_hh"), crow=self.gate_perm_i32),
                  Gemm(dgT, X, L.view(g, "lstm.weight_ih"), crow=self.gate_perm_i32)]
        x_job = Gemm(self.dgates, pk["w_ih"], self.dX)                # (N, D) bf16
        bias_done = self._lstm_bwd(dh)
        splits = self._group_splits(w_jobs, x_job)
        if splits:
            # weight gradients and dX share one grid (gemm_group_kernel), longest K first
            gemm_group([w_jobs[2], w_jobs[1], w_jobs[0], x_job], splits, self.gg_ws, self.gg_tickets)
        else:
            gemm(w_jobs[2], w_jobs[1], w_jobs[0])
            gemm(x_job)
        # bias grads: column sums of dgates, packed -> torch gate order, into both biases (fused
        # into the tagged BPTT kernel when it ran)
        if not bias_done:
            check(k.r2_colsum_bf16(ptr(self.dgates), N, G, ptr(self.gate_perm_i32),
                                   ptr(L.view(g, "lstm.bias_ih")), ptr(L.view(g, "lstm.bias_hh")),
                                   ptr(self.gs_ws), ptr(self.gs_ticket[32:]), s), "colsum")
        self._dX = self.dX

    def _group_splits(self, w_jobs, x_job):
        """K splits of the grouped post-BPTT launch ([dW_ih, dW_hh, dW_head1, dX]) or None for
        separate launches.  ``learner.bwd_gemm``: "group" = no split,
        "group:a,b,c,d" = explicit splits, "separate".  Needs every K % 64 == 0."""
        mode = self.cfg.learner.bwd_gemm
        if not mode.startswith("group"):
            return None
        splits = [int(v) for v in mode.split(":")[1].split(",")] if ":" in mode else [1, 1, 1, 1]
        probs = [w_jobs[2], w_jobs[1], w_jobs[0], x_job]
        if len(splits) != 4 or any(p.a.shape[1] % 64 for p in probs):
            return None
        need = group_ws_bytes(probs, splits)
        if getattr(self, "gg_ws", None) is None or self.gg_ws.numel() * 4 < need:
            if torch.cuda.is_current_stream_capturing():
                return None
            self.gg_ws = torch.zeros(need // 4 + 1, dtype=torch.float32, device=self.device)
            self.gg_tickets = torch.zeros(1024, dtype=torch.int32, device=self.device)
        return splits

    def _lstm_bwd(self, dh: torch.Tensor) -> bool:
        """BPTT over the learning window: dgates (Ll, B, G) from dh (Ll, B, H), plus the head
        gradient reduction (``self._hg_job``) on the tagged launch's idle workgroups or on its own.
        Returns True when the kernel also produced the LSTM bias gradients (tagged BPTT)."""
        k = kernels()
        s = stream_handle()
        B, T, Lb, H, pk = self.B, self.T, self.Lb, self.layout.H, self.pk
        lc, L, g = self.cfg.learner, self.layout, self.grad
        if lc.lstm_impl == "persistent" and lc.lstm_handoff == "tagged":
            base = [ptr(dh), ptr(self.gates), ptr(self.cseq["on"]), ptr(self.c0["on"]),
                    ptr(pk["w_hhT"]), ptr(self.dgates), B, T, Lb, H, ptr(self.ctr), ptr(self.err),
                    ptr(self.ring_b), ptr(self.bias_ws), ptr(self.gate_perm_i32),
                    ptr(L.view(g, "lstm.bias_ih")), ptr(L.view(g, "lstm.bias_hh"))]
            rc = k.r2_lstm_bwd_tag(*base, *self._hg_job, s)
            if rc in (-6, -10):   # not enough idle workgroups for the side job: recurrence alone
                rc = k.r2_lstm_bwd_tag(*base, *([0] * 11), s)
            if rc != -3:          # -3: grid too large for one workgroup per CU
                if rc < 0:
                    check(rc, "lstm_bwd_tag")
                if not rc & 1:
                    check(k.r2_head_grads(*self._hg_job, s), "head_grads")
                return True
        check(k.r2_head_grads(*self._hg_job, s), "head_grads")
        if lc.lstm_impl == "persistent":
            check(k.r2_lstm_bwd_persist(ptr(dh), ptr(self.gates), ptr(self.cseq["on"]),
                                        ptr(self.c0["on"]), ptr(pk["w_hhT"]), ptr(self.slab_p),
                                        ptr(self.dgates), B, T, Lb, H, ptr(self.ctr), ptr(self.err),
                                        s), "lstm_bwd_persist")
        else:
            self.dc.zero_()
            check(k.r2_lstm_bwd(ptr(dh), ptr(self.gates), ptr(self.cseq["on"]), ptr(self.c0["on"]),
                                ptr(pk["w_hhT"]), ptr(self.slab0), ptr(self.slab1), ptr(self.dc),
                                ptr(self.dgates), B, T, Lb, H, s), "lstm_bwd")
        return False

    def _relu_mask(self, grad: torch.Tensor, act: torch.Tensor) -> torch.Tensor:
        """grad * (act > 0) for two tensors with the same (channels-last) memory layout."""
        cl = torch.channels_last
        if grad.is_contiguous(memory_format=cl) and act.is_contiguous(memory_format=cl):
            out = torch.empty_like(grad)
            check(kernels().r2_relu_mask_bf16(ptr(grad), ptr(act), ptr(out), grad.numel(),
                                              stream_handle()), "relu_mask")
            return out
        return grad * (act > 0)

    def _backward_torso(self, defer_reduce: bool = False):
        """Conv-torso backward into self.grad.  ``defer_reduce`` (split precision, world 1): the
        per-workgroup gradient slabs are left for the optimizer launch, which sums them
        (r2_rmsprop_pack_slab); the torso entries of self.grad are written there."""
        self._torso_deferred = False
        if self.sp_lib:
            B, Lb, T = self.B, self.Lb, self.T
            torso_backward_library_sp(self.replay.frames, self.rows[Lb * B: T * B], self.layout,
                                      self.master, self.cfg.env, self.cfg.model, self.tdims[1],
                                      self.dX, self.dX_lo, self.X_on[Lb * B: T * B], self.act1,
                                      self.act2, self.grad)
            return
        if self.sp:
            B, Lb, T = self.B, self.Lb, self.T
            pk, pkl = self.pk, self.pk_lo
            check(kernels().r2_torso_bwd_sp(
                ptr(self.replay.frames), ptr(self.rows[Lb * B: T * B]), self.Ll * B, ptr(self.act1),
                ptr(self.act1_lo), ptr(self.act2), ptr(self.act2_lo), ptr(self.dX), ptr(self.dX_lo),
                ptr(self.X_on[Lb * B: T * B]), ptr(pk["conv3_dg"]), ptr(pkl["conv3_dg"]),
                ptr(pk["conv2_dg"]), ptr(pkl["conv2_dg"]), ptr(self._tb_slab), self._tb_grid,
                ptr(self._tb_dst), ptr(self._tb_scale),
                0 if defer_reduce else ptr(self.grad), stream_handle()), "torso_bwd_sp")
            self._torso_deferred = defer_reduce
            return
        if self.cfg.learner.torso_bwd == "fused" and self.fwd_geom is not None:
            self._backward_torso_fused()
        else:
            self._backward_torso_library()

    def _backward_torso_fused(self):
        """One fused HIP kernel (csrc/kernels/torso_bwd.hip, Atari or DMLab geometry) + slab
        reduction into self.grad."""
        B, Lb, T = self.B, self.Lb, self.T
        N = self.Ll * B
        pk = self.pk
        fr = self.replay.frames
        check(kernels().r2_torso_bwd_geom(ptr(fr), fr.stride(0) * fr.element_size(),
                                          ptr(self.rows[Lb * B: T * B]), N,
                                          ptr(self.act1), ptr(self.act2), ptr(self._dX),
                                          ptr(self.X_on[Lb * B: T * B]), ptr(pk["conv3_dg"]),
                                          ptr(pk["conv2_dg"]), ptr(self._tb_slab), self._tb_grid,
                                          ptr(self._tb_dst), ptr(self._tb_scale), ptr(self.grad),
                                          *self.fwd_geom, stream_handle()), "torso_bwd")

    def _backward_torso_library(self):
        """Conv backward (library kernels) from the activations saved by the torso kernel.
        Everything is channels-last so the library picks its NHWC kernels with no transposes."""
        k = kernels()
        s = stream_handle()
        B, Lb, Ll, T = self.B, self.Lb, self.Ll, self.T
        L, g = self.layout, self.grad
        N = Ll * B
        cl = torch.channels_last
        cin, dims = self.tdims
        c1, c2, c3 = self.cfg.model.conv_channels
        (h1, w1_), (h2, w2_), (h3, w3_) = dims
        fh, fw = self.cfg.env.frame_h, self.cfg.env.frame_w
        out3 = self.X_on[Lb * B: T * B]
        g3 = torch.empty_like(self._dX)
        check(k.r2_relu_mask_bf16(ptr(self._dX), ptr(out3), ptr(g3), g3.numel(), s), "relu_mask")
        g3 = g3.view(N, c3, h3, w3_).contiguous(memory_format=cl)
        a2 = self.act2.view(N, h2, w2_, c2).permute(0, 3, 1, 2)
        a1 = self.act1.view(N, h1, w1_, c1).permute(0, 3, 1, 2)
        m = self.master
        w3 = L.view(m, "vis_layers.4.weight").to(torch.bfloat16)
        w2 = L.view(m, "vis_layers.2.weight").to(torch.bfloat16)
        w1 = L.view(m, "vis_layers.0.weight").to(torch.bfloat16)
        cb = torch.ops.aten.convolution_backward
        d2, dw3, db3 = cb(g3, a2, w3, [c3], [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                          [True, True, True])
        g2 = self._relu_mask(d2, a2)
        d1, dw2, db2 = cb(g2, a1, w2, [c2], [2, 2], [0, 0], [1, 1], False, [0, 0], 1,
                          [True, True, True])
        g1 = self._relu_mask(d1, a1)
        rows = self.rows[Lb * B: T * B]
        if self.fused_torso:
            check(k.r2_frames_to_bf16_nhwc(ptr(self.replay.frames), ptr(rows), N,
                                           ptr(self.frames_bf), s), "frames_to_bf16_nhwc")
        else:   # exact 0..255 values; the 1/255 is applied to dW1 in fp32 below
            gather_frames_nhwc(self.replay.frames, rows, cin, fh, fw, out=self.frames_bf)
        fr = self.frames_bf.view(N, fh, fw, cin).permute(0, 3, 1, 2)
        _, dw1, db1 = cb(g1, fr, w1, [c1], [4, 4], [0, 0], [1, 1], False, [0, 0], 1,
                         [False, True, True])
        if not self.fused_torso:
            dw1 = dw1.float() * (1.0 / 255)
        L.view(g, "vis_layers.4.weight").copy_(dw3)
        L.view(g, "vis_layers.4.bias").copy_(db3)
        L.view(g, "vis_layers.2.weight").copy_(dw2)
        L.view(g, "vis_layers.2.bias").copy_(db2)
        L.view(g, "vis_layers.0.weight").copy_(dw1)
        L.view(g, "vis_layers.0.bias").copy_(db1)

    def _update(self):
        assert getattr(self, "_pack_deferred", None) is None, \
            "a deferred weight repack was never run (_update without _priorities after it)"
        k = kernels()
        s = stream_handle()
        lc, L = self.cfg.learner, self.layout
        n = L.padded
        gscale = 1.0 / self.world
        clip = 0
        if lc.grad_clip > 0:
            check(k.r2_sumsq(ptr(self.grad), n, ptr(self.clip_buf), s), "sumsq")
            clip = ptr(self.clip_buf)
        if lc.optimizer == "adam":
            check(k.r2_adam(ptr(self.master), ptr(self.grad), ptr(self.opt_a), ptr(self.opt_b), n,
                            float(lc.lr), float(lc.adam_betas[0]), float(lc.adam_betas[1]),
                            float(lc.eps), gscale, ptr(self.replay.step), clip,
                            float(lc.grad_clip), s), "adam")
        elif self._fold_tq is not None and getattr(self, "_torso_deferred", False):
            # + the torso slab reduction (its first workgroups; _backward_torso left the slabs)
            check(k.r2_rmsprop_pack_slab(ptr(self.master), ptr(self.grad), ptr(self.opt_a),
                                         ptr(self.opt_b), n, float(lc.lr), float(lc.rms_alpha),
                                         float(lc.eps), gscale, ptr(self.row_dst4), ptr(self.bf),
                                         ptr(self.bf_t), L.bf_numel if self.sp else 0,
                                         ptr(self.target), ptr(self.replay.step),
                                         self._baked_interval(), ptr(self._tb_slab), self._tb_grid,
                                         int(kernels().r2_torso_bwd_slab_floats()), ptr(self._tb_dst),
                                         ptr(self._tb_scale), self._fold_tq, s), "rmsprop_pack_slab")
            self._pack_step(self._baked_interval(), s, rows_done=True)
            return
        elif self.row_dst4 is not None:
            # the update writes the row packs (w_ih / w_hh / head1) and, when due, the target
            # master itself; the pack launch below gathers the rest
            check(k.r2_rmsprop_pack(ptr(self.master), ptr(self.grad), ptr(self.opt_a),
                                    ptr(self.opt_b), n, float(lc.lr), float(lc.rms_alpha),
                                    float(lc.eps), gscale, clip, float(lc.grad_clip),
                                    ptr(self.row_dst4), ptr(self.bf), ptr(self.bf_t),
                                    L.bf_numel if self.sp else 0, ptr(self.target),
                                    ptr(self.replay.step), self._baked_interval(), s),
                  "rmsprop_pack")
            self._pack_step(self._baked_interval(), s, rows_done=True)
            return
        else:
            check(k.r2_rmsprop_centered(ptr(self.master), ptr(self.grad), ptr(self.opt_a),
                                        ptr(self.opt_b), n, float(lc.lr), float(lc.rms_alpha),
                                        float(lc.eps), gscale, clip, float(lc.grad_clip), s),
                  "rmsprop")
        # one launch: online repack + target sync on device when (step+1) % interval == 0
        # (learner.py:107-108) with the target packs written only then
        self._pack_step(self._baked_interval(), s)

    def _priorities(self, end: bool = True):
        rp = self.replay
        deferred = getattr(self, "_pack_deferred", None)
        self._pack_deferred = None
        if deferred is not None:
            head, tail = self._pack_args(*deferred)
            if end and rp.prio_tail(self.starts, self.B, self.Lb, self.T, end, pack=head + tail):
                return
            # refused (shape): the repack as its own launch, then the separate tail
            check(kernels().r2_pack_step(*head, ptr(rp.step), *tail, stream_handle()), "pack_step")
        if self.cfg.replay.fused_prio_tail and rp.prio_tail(self.starts, self.B, self.Lb, self.T, end):
            return
        rp.refresh_sequences(self.starts, self.B, self.Lb, self.T)
        if self.cfg.replay.fused_tree_tail and rp.update_tree_and_end_step(end):
            return
        rp.update_tree()
        if end:
            rp.step_end()

    # ------------------------------------------------------------------ public API
    def _sync(self):
        if getattr(self, "_gsync", None) is None:
            from ..parallel.grad_sync import GradSync
            self._gsync = GradSync(self.grad, self.world, self.pg, self.cfg.dist.grad_dtype,
                                   use_stream=self.cfg.dist.overlap_allreduce, force=self.dp)
        return self._gsync

    def _seg_core(self):
        self._forward_loss()
        self._backward_core()

    # DP with global sampling: the sampled batch's shard stats are all-gathered between the
    # sampling launch and the rest of the forward
    def _seg_sample(self):
        self._sample()

    def _seg_core_rest(self):
        self._forward_rest()
        self._backward_core()

    def _seg_fwd_head(self):       # DP global sampling: everything before the TD (gather in flight)
        self._forward_rest(tail=False)

    def _seg_core_tail(self):      # ... and from the heads / TD on (gathered stats joined)
        self._forward_tail()
        self._backward_core()

    def _seg_torso(self):
        # the update that follows (same segment) sums the slabs itself when folded
        self._backward_torso(defer_reduce=self._fold_tq is not None)

    def _seg_tail(self):
        self._update()
        self._priorities()

    def _single_body(self, timer=None):
        """The world == 1 step as stream operations (eager or captured).  (Running the priority
        refresh + tree repair on a side stream beside the BPTT was measured neutral and removed:
        profiles/r03_prio_side_stream_ab.txt.)"""
        import contextlib
        ph = timer.phase if timer is not None else (lambda name: contextlib.nullcontext())
        with ph("forward+td"):
            self._forward_loss()
        with ph("backward_core"):
            self._backward_core()
        with ph("backward_torso"):
            self._seg_torso()
        with ph("update"):
            self._update()
        with ph("priorities"):
            self._priorities()

    # DP (world > 1): the priority refresh + tree repair need only the forward's TD errors, so
    # they run while the torso bucket is all-reduced; the update and the step counter follow
    def _seg_prio(self):
        self._priorities(end=False)

    def _seg_update(self):
        self._update()
        self.replay.step_end()

    def step_eager(self, timer=None):
        """One step without the graph.  ``timer``: optional utils.profiling.PhaseTimer -- every
        phase is bracketed by HIP events and a roctx range (bench.py --profile-phases)."""
        import contextlib
        L = self.layout
        ph = timer.phase if timer is not None else (lambda name: contextlib.nullcontext())
        if self.hoist:     # (no per-phase timer: the step's phases overlap on two streams)
            g, self.graph = self.graph, None
            try:
                self._hoist_step()
            finally:
                self.graph = g
            return
        if not self.dp:
            self._single_body(timer)
            self.steps_done += 1
            return
        with ph("forward+td"):
            self._forward_loss()      # (DP global sampling: includes the stats all-gather)
        with ph("backward_core"):
            self._backward_core()
        self._sync().start(0, L.torso_offset)        # core bucket: overlaps the conv backward
        with ph("backward_torso"):
            self._seg_torso()
        self._sync().start(L.torso_offset, L.padded)  # torso bucket: overlaps the priority tail
        with ph("priorities"):
            self._seg_prio()
        with ph("allreduce_wait"):
            self._sync().finish()
        with ph("update"):
            self._seg_update()
        self.steps_done += 1

    def capture(self, warmup: int = 2):
        """Capture the step into HIP graphs.  world == 1: one graph for the whole step.
        world > 1: four graphs (core fwd/bwd | conv bwd | priorities | update) with the two
        bucket all-reduces issued between them on the communication stream; with global
        sampling the core graph is split after the sampling launch and again before the heads /
        TD (six graphs): the 12-byte shard-stats all-gather runs on its own stream beside the
        torso / x-projection / LSTM graph and is joined before the TD."""
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step_eager()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self.graphs = []
        self._one_dp_graph = False
        if self.hoist:
            # the hoisted step's graph variants: (sample set, sampled by the previous step or
            # not, target sync due) -- all eight captured now, none inside a timed loop
            self._hgraphs, self._hpool = {}, None
            cur, due = self._cur, getattr(self, "_hoist_due", False)
            for key in [(p, i, d) for p in (0, 1) for i in ("H", "P") for d in (False, True)]:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self._hpool):
                    self._hoist_body(*key)
                if self._hpool is None:
                    self._hpool = g.pool()
                self._hgraphs[key] = g
            # runs of graph_chunk steps starting at an even step, none due, previous step sampled
            # (run_steps): one graph, so the inter-replay boundary is paid once per chunk
            self._cgraph = None
            m = self._chunk_len()
            if m > 1:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self._hpool):
                    for j in range(m):
                        self._hoist_body(j & 1, "H", False)
                self._cgraph = g
                _graph_upload(g)
            self._use_set(cur)
            self._hoist_due = due
            torch.cuda.synchronize(self.device)
            self.graph = True
            return
        one = self.cfg.dist.graph_collectives and (self.world == 1 or self.cfg.dist.graph_collectives_multi)
        if self.dp:
            # the segment graphs first; the whole DP step as ONE graph (collectives captured on
            # their side streams) replaces them after dist.one_graph_warm steps and, at world > 1,
            # a validation window (parallel/graph_rollout.py)
            from ..parallel.graph_rollout import GraphRollout
            dc = self.cfg.dist
            self._rollout = GraphRollout(self.pg, self.rank, self.world,
                                         enabled=one and self._pg_backend() == "nccl",
                                         warm=int(dc.one_graph_warm), validate=int(dc.one_graph_validate),
                                         device=self.device)
        if self.dp:
            segs = [self._seg_core, self._seg_torso, self._seg_prio, self._seg_update]
            if self.dp_global:
                segs = [self._seg_sample, self._seg_fwd_head, self._seg_core_tail] + segs[1:]
        else:
            segs = [self._single_body]
        pool = None
        for fn in segs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode=self._capture_mode()):
                fn()
            pool = g.pool()
            self.graphs.append(g)
        torch.cuda.synchronize(self.device)
        self.graph = True

    def _capture_mode(self) -> str:
        """Graph capture error mode: with a process group the RCCL watchdog thread polls the events
        of earlier collectives while this thread captures, which global mode turns into a capture
        error (hipErrorStreamCaptureUnsupported on the watchdog, seen as a flaky forced-DP test);
        thread-local mode confines the capture rules to this thread."""
        return "thread_local" if self.dp else "global"

    def _pg_backend(self) -> str:
        """Backend of the DP process group (only RCCL collectives can be graph-captured; gloo
        ones -- CPU tests, ranks sharing a GPU -- stay between segment graphs)."""
        import torch.distributed as dist
        try:
            return str(dist.get_backend(self.pg))
        except (RuntimeError, ValueError):
            return ""

    def _dp_step_body(self):
        """The DP step as stream operations (capturable): segments in order, the collectives on
        their side streams with event fork / join -- what ``step`` issues between the segment
        graphs."""
        L = self.layout
        if self.dp_global:
            self._seg_sample()
            main = torch.cuda.current_stream(self.device)
            if getattr(self, "_gather_stream", None) is None:
                self._gather_stream = torch.cuda.Stream(device=self.device)
            gs = self._gather_stream
            gs.wait_stream(main)
            with torch.cuda.stream(gs):
                self._gather_dp()
            self._seg_fwd_head()
            main.wait_stream(gs)
            self._seg_core_tail()
        else:
            self._seg_core()
        self._sync().start(0, L.torso_offset)
        self._seg_torso()
        self._sync().start(L.torso_offset, L.padded)
        self._seg_prio()
        self._sync().finish()
        self._seg_update()

    def _capture_one_dp(self) -> None:
        """The whole DP step in ONE graph: the bucket all-reduces and the shard-stats all-gather
        are captured on their side streams (fork / join as graph edges), so the ~15 us gap of
        every segment boundary disappears."""
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.graphs[0].pool() if self.graphs else None,
                              capture_error_mode=self._capture_mode()):
            self._dp_step_body()
        torch.cuda.synchronize(self.device)
        self._one_graph = g
        self._one_dp_graph = True

    def _dp_checksum(self) -> torch.Tensor:
        """A fingerprint of this rank's weights (0-d float64, on the device): equal on every rank
        while the ranks stay in lock-step."""
        return self.master.double().sum() + 3.0 * self.target.double().sum()

    def _dp_repair(self) -> None:
        """After a one-graph validation mismatch: every rank takes rank 0's weights and optimizer
        state, and re-packs its kernel layouts."""
        import torch.distributed as dist
        src = dist.get_global_rank(self.pg, 0) if hasattr(dist, "get_global_rank") else 0
        for t in (self.master, self.target, self.opt_a, self.opt_b):
            dist.broadcast(t, src=src, group=self.pg)
        self._pack(always=True)
        self._one_dp_graph = False

    def _dp_rollout_after_step(self) -> None:
        ro = getattr(self, "_rollout", None)
        if ro is None:
            return
        if ro.validating():
            if ro.record(self._dp_checksum(), self.err, self.steps_done) is False:
                self._dp_repair()
        elif ro.want_promote(self.steps_done):
            err = None
            try:
                self._capture_one_dp()
            except Exception as e:   # noqa: BLE001 -- the runtime refused the capture
                err = "%s: %s" % (type(e).__name__, str(e).splitlines()[0][:120] if str(e) else "")
                self._one_graph, self._one_dp_graph = None, False
                # host-side step state a half-captured body may have left behind
                self._pack_deferred = None
                self._gsync = None
                torch.cuda.synchronize(self.device)
            if ro.agree(err is None):
                ro.promoted()
            else:
                self._one_graph, self._one_dp_graph = None, False
                ro.refused(err or "on another rank")

    def dp_graph_label(self) -> Optional[str]:
        """How the DP step is replayed (bench.py JSON): segment graphs, the one graph (validated
        or still validating), or the fallback after a mismatch; None without DP."""
        if not self.dp:
            return None
        ro = getattr(self, "_rollout", None)
        return ro.label() if ro is not None else "eager"

    def step(self):
        if self.hoist and self.graph:
            self._hoist_step()
            return
        if not self.graph:
            self.step_eager()
            return
        if not self.dp:
            self.graphs[0].replay()
        elif getattr(self, "_rollout", None) is not None and self._rollout.mode == "one":
            self._one_graph.replay()
            self.steps_done += 1
            self._dp_rollout_after_step()
            return
        else:
            L = self.layout
            if self.dp_global:
                g_sample, g_fwd, g_core, g_torso, g_prio, g_update = self.graphs
                g_sample.replay()
                # the shard-stats all-gather runs on its own stream beside the torso / LSTM graph
                main = torch.cuda.current_stream(self.device)
                if getattr(self, "_gather_stream", None) is None:
                    self._gather_stream = torch.cuda.Stream(device=self.device)
                gs = self._gather_stream
                gs.wait_stream(main)
                with torch.cuda.stream(gs):
                    self._gather_dp()
                g_fwd.replay()
                main.wait_stream(gs)
            else:
                g_core, g_torso, g_prio, g_update = self.graphs
            g_core.replay()
            self._sync().start(0, L.torso_offset)
            g_torso.replay()
            self._sync().start(L.torso_offset, L.padded)
            g_prio.replay()
            self._sync().finish()
            g_update.replay()
            self.steps_done += 1
            self._dp_rollout_after_step()
            return
        self.steps_done += 1

    def dp_imbalance(self) -> float:
        """W * sum_k (S_k / S)^2 of the last step's gathered shard totals: the variance inflation
        of the fixed-B shard-ratio sampling over one merged replay (parallel/sharded_replay.py;
        1.0 = balanced shards).  One D2H read; 1.0 without DP global sampling."""
        if not self.dp_global:
            return 1.0
        from ..parallel.sharded_replay import imbalance_factor
        return float(imbalance_factor(self.dp_recv.view(self.world, 3)))

    def loss_value(self) -> float:
        return float(self.loss.item())

    @torch.no_grad()
    def diagnostics(self) -> Dict[str, float]:
        """Learner diagnostics of the last step (the reference prints only a step
        count, ``/root/reference/learner.py:57-59``): loss, Q(s, .) of the online net over the
        learning rows (mean, mean of max_a, max), |TD error| (mean, max: the priority input),
        IS weights (mean, min), the replay's sampleable sequences, fill and priority total (the
        sum tree's root).  One D2H copy; call at log cadence, not per step."""
        rp = self.replay
        N = self.Ll * self.B
        q = self.q_on[:N]
        td = self.td_abs[:N]
        root = rp.tree[int(rp.tree_offs[-1]): int(rp.tree_offs[-1]) + 1]
        v = torch.stack([self.loss.reshape(()), q.mean(), q.max(1).values.mean(), q.max(),
                         td.mean(), td.max(), self.is_w.mean(), self.is_w.min(),
                         root.reshape(()).float(), rp.n_valid.reshape(()).float()]).tolist()
        keys = ("loss", "q_mean", "q_max_a_mean", "q_max", "td_abs_mean", "td_abs_max",
                "is_w_mean", "is_w_min", "priority_sum", "n_valid")
        out = dict(zip(keys, v))
        out["replay_fill"] = rp.size / rp.capacity
        return out

    def error_word(self) -> int:
        """The persistent kernels' error word (non-zero: a bounded hand-off spin timed out, so the
        step's recurrent state is garbage; bit 30: the priority tail's grid barrier timed out, so
        the sum tree missed a repair).  One or two D2H reads."""
        w = int(self.err.item())
        ps = getattr(self.replay, "prio_sync", None)
        if ps is not None and int(ps[3].item()) != 0:
            w |= 1 << 30
        return w

    def check_errors(self) -> None:
        """Raise if a persistent kernel's bounded spin timed out (hand-off failure)."""
        w = self.error_word()
        if w & (1 << 30):
            raise RuntimeError("priority tail kernel reported a grid-barrier timeout")
        if w != 0:
            raise RuntimeError("persistent LSTM kernel reported a hand-off timeout")
