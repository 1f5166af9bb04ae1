"""CPU actor -> HBM replay ingest throughput (shared-memory rings, zero-copy DMA, device scatter).

N producer processes each push K records of R rows (the reference's transport unit: an actor's
local replay, 5000 rows = 161 MB at the Atari schema) into their own ring; the learner process
drains them with ``engine.ingest.HBMIngestor``.  Reference: loading a 5000-row file takes 1.23 s
(``replay_memory.py:155-173``), i.e. ~4.1k rows/s.

    python tools/bench_ingest.py --producers 4 --records 6 --rows 5000
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time
import uuid

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def _synthetic_record(rows, seed, H=256):
    from pytorch_r2d2_amd.parallel.trajectory import pack_rows
    rng = np.random.default_rng(seed)
    m = {
        "state": rng.integers(0, 256, (rows, 4, 84, 84), dtype=np.uint8),
        "hs_cs": rng.normal(size=(rows, 2 * H)).astype(np.float32),
        "target_hs_cs": rng.normal(size=(rows, 2 * H)).astype(np.float32),
        "action": rng.integers(0, 6, (rows, 1)).astype(np.int8),
        "reward": rng.normal(size=(rows, 1)).astype(np.float32),
        "done": (rng.random((rows, 1)) < 0.003).astype(np.float32),
        "stack_count": np.ones(rows, dtype=np.int8),
        "priority": rng.random(rows).astype(np.float32) + 0.1,
        "sequence_priority": np.zeros(rows, dtype=np.float32),
        "is_seq_start": np.zeros(rows, dtype=np.uint8),
    }
    st = (np.arange(rows) % 40 == 0) & (np.arange(rows) <= rows - 80)
    m["is_seq_start"][:] = st
    m["sequence_priority"][:] = np.where(st, rng.random(rows) + 0.5, 0).astype(np.float32)
    return pack_rows(m)


def _producer(name, ring_bytes, records, rows, seed):
    from pytorch_r2d2_amd.runtime import ShmRing
    ring = ShmRing(name, ring_bytes, create=False)
    rec = _synthetic_record(rows, seed)
    for _ in range(records):
        while not ring.push(rec):
            time.sleep(0.0005)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--producers", type=int, default=4)
    ap.add_argument("--records", type=int, default=6)
    ap.add_argument("--rows", type=int, default=5000)
    ap.add_argument("--no-register", action="store_true", help="pinned bounce buffer instead")
    a = ap.parse_args()
    import torch
    from pytorch_r2d2_amd.config import get_config
    from pytorch_r2d2_amd.engine.ingest import HBMIngestor
    from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay
    dev = torch.device("cuda")
    cfg = get_config("atari57")
    P = a.producers
    rp = HBMReplay(cfg, dev, capacity=P * 4 * a.rows, n_subrings=P)
    ring_bytes = int(2.2 * len(_synthetic_record(8, 0)) / 8 * a.rows) + (1 << 20)
    names = [f"/r2d2_bi_{uuid.uuid4().hex[:6]}_{i}" for i in range(P)]
    ing = HBMIngestor(rp, names, ring_bytes=ring_bytes, register=not a.no_register)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_producer, args=(n, ring_bytes, a.records, a.rows, i))
             for i, n in enumerate(names)]
    for p in procs:
        p.start()
    want = P * a.records * min(a.rows, rp.cap_e)
    t0 = None
    deadline = time.time() + 600
    while ing.rows < want and time.time() < deadline:
        got = ing.poll()
        if got and t0 is None:
            t0 = time.perf_counter()
            rows0, bytes0 = ing.rows - got, ing.bytes - ing.bytes   # noqa: F841
        if not got:
            time.sleep(0.0002)
    ing._release_done(wait=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for p in procs:
        p.join(30)
    first = min(a.rows, rp.cap_e)
    rows = ing.rows - first            # the first record starts the clock
    dt = t1 - t0
    rec = {"metric": "ingest_rows_per_s", "value": round(rows / dt, 1), "unit": "rows/s",
           "GB_per_s": round((ing.bytes * rows / max(ing.rows, 1)) / dt / 1e9, 2),
           "producers": P, "records": ing.records, "rows_per_record": a.rows,
           "zero_copy": all(b is not None for b in ing.registered),
           "reference_rows_per_s": round(5000 / 1.23, 1),
           "vs_reference": round(rows / dt / (5000 / 1.23), 1),
           "n_valid": int(rp.n_valid.item()), "ingest_err": int(rp.ingest_err.item())}
    print(json.dumps(rec), flush=True)
    ing.close()


if __name__ == "__main__":
    main()
