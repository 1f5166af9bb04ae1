"""Collective micro-benchmark for the learner's communication pattern.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_collectives.py
    python tools/bench_collectives.py --backend gloo --world 2      # CPU rehearsal (spawns ranks)

Message sizes are the learner's: the gradient buckets of the flat fp32 buffer (core = LSTM +
head, ~8.0 MB; torso = conv, ~0.14 MB; the whole 8.15 MB), their bf16-compressed halves, the
weight broadcast (8.15 MB from rank 0) and the shard-total all-gather of the sharded replay
(8 floats).  Reports per op: mean latency and the algorithm / bus bandwidth nccl-tests style
(all_reduce busbw = algbw * 2 (p-1)/p, broadcast busbw = algbw, all_gather (p-1)/p).  On
MI355X xGMI (7 links x ~153 GB/s per GPU) an 8 MB all-reduce is per-link bound; RCCL stripes
the ring channels over the links.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GRAD_PARAMS = 2_037_095        # reference model.py parameter count
TORSO_PARAMS = 8_192 + 32 + 16_384 + 32 + 9_216 + 32


def _cases(world):
    core = GRAD_PARAMS - TORSO_PARAMS
    return [
        ("all_reduce_core_fp32", "all_reduce", core, torch.float32),
        ("all_reduce_torso_fp32", "all_reduce", TORSO_PARAMS, torch.float32),
        ("all_reduce_all_fp32", "all_reduce", GRAD_PARAMS, torch.float32),
        ("all_reduce_all_bf16", "all_reduce", GRAD_PARAMS, torch.bfloat16),
        ("broadcast_weights_fp32", "broadcast", GRAD_PARAMS, torch.float32),
        ("all_gather_shard_totals", "all_gather", 8, torch.float32),
    ]


def run(iters: int, warmup: int, device: torch.device) -> dict:
    world, rank = dist.get_world_size(), dist.get_rank()
    out = {"metric": "collective_latency", "world": world, "backend": dist.get_backend(),
           "device": str(device)}
    sync = (lambda: torch.cuda.synchronize(device)) if device.type == "cuda" else (lambda: None)
    for name, op, n, dt in _cases(world):
        x = torch.ones(n, dtype=dt, device=device)
        outs = [torch.empty(n, dtype=dt, device=device) for _ in range(world)]

        def once():
            if op == "all_reduce":
                dist.all_reduce(x)
            elif op == "broadcast":
                dist.broadcast(x, src=0)
            else:
                dist.all_gather(outs, x)

        for _ in range(warmup):
            once()
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            once()
        sync()
        dt_s = (time.perf_counter() - t0) / iters
        tt = torch.tensor([dt_s], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt_s = float(tt.item())
        nbytes = n * x.element_size()
        algbw = nbytes / dt_s / 1e9
        factor = {"all_reduce": 2 * (world - 1) / world, "broadcast": 1.0,
                  "all_gather": (world - 1) / world}[op]
        out[name] = {"bytes": nbytes, "us": round(dt_s * 1e6, 2), "algbw_GBs": round(algbw, 2),
                     "busbw_GBs": round(algbw * factor, 2)}
    return out


def _worker(rank, world, port, backend, iters, warmup):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    main_body(backend, iters, warmup)


def main_body(backend, iters, warmup):
    from pytorch_r2d2_amd.parallel.dist import init_distributed, shutdown
    info = init_distributed(backend=backend,
                            device_type="cpu" if backend == "gloo" else None)
    if info.world <= 1:
        print(json.dumps({"metric": "collective_latency", "world": 1, "skipped": "single rank"}))
        return None
    res = run(iters, warmup, info.device)
    if info.is_main:
        print(json.dumps(res), flush=True)
    shutdown()
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--world", type=int, default=0,
                    help="spawn this many local ranks (no torchrun); CPU/gloo rehearsal")
    args = ap.parse_args(argv)
    if args.world > 1 and "WORLD_SIZE" not in os.environ:
        import socket
        import torch.multiprocessing as mp
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        mp.spawn(_worker, args=(args.world, port, args.backend, args.iters, args.warmup),
                 nprocs=args.world, join=True)
        return
    main_body(args.backend, args.iters, args.warmup)


if __name__ == "__main__":
    main()
