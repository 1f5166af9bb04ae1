"""Where the persistent LSTM launches spend the time before their first step (fp32 bench config,
eager engine steps).  Forward: per-workgroup stamps of lstm_fwd_tag_kernel
(r2_lstm_fwd_set_stamps: start, XCD rendezvous done, compute loop entry, end); BPTT: the
PTBArgs::dbg words of lstm_bwd_tag_kernel (start [0], end [1], role [2], rendezvous done [6],
loop entry [7]).  us from each launch's first workgroup start (s_memrealtime, 100 MHz).

    python tools/lstm_startup_probe.py [key=value ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_r2d2_amd.config import get_config  # noqa: E402
from pytorch_r2d2_amd.engine.learner_engine import LearnerEngine  # noqa: E402
from pytorch_r2d2_amd.engine.replay_hbm import HBMReplay  # noqa: E402
from pytorch_r2d2_amd.ops._lib import kernels, ptr  # noqa: E402

DEV = torch.device("cuda")


def med(x):
    return round(float(np.median(x)) / 100.0, 2)


def main(reps: int = 3, overrides=()):
    ov = {"seed": 1234, "learner.use_graph": False}
    for kv in overrides:        # key=value config overrides (ints / floats / bools / strings)
        key, v = kv.split("=", 1)
        ov[key] = {"True": True, "False": False}.get(v, int(v) if v.lstrip("-").isdigit() else v)
    cfg = get_config("atari57", **ov)
    replay = HBMReplay(cfg, DEV, capacity=200_000)
    replay.fill_synthetic(episode_len=400, seed=0)
    eng = LearnerEngine(cfg, replay, DEV)
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    k = kernels()
    if not k.r2_lstm_probes():
        raise SystemExit("the LSTM stamp hooks are compiled out: rebuild with "
                         "R2D2_PROBES=1 python -m pytorch_r2d2_amd._build")
    for _ in range(reps):
        fs = torch.zeros(4 * 512, dtype=torch.int64, device=DEV)
        dbg = torch.zeros(4096, dtype=torch.int64, device=DEV)
        k.r2_lstm_fwd_set_stamps(ptr(fs))
        k.r2_lstm_persist_set_debug(ptr(dbg))
        eng.step()
        torch.cuda.synchronize()
        k.r2_lstm_fwd_set_stamps(None)
        k.r2_lstm_persist_set_debug(None)
        f = fs.view(-1, 4).cpu().numpy()
        f = f[f[:, 0] > 0]
        t0 = f[:, 0].min()
        b = dbg.cpu().numpy()[:2048].reshape(256, 8)
        rec = b[b[:, 2] == 1]
        u0 = b[b[:, 2] > 0, 0].min()
        print(json.dumps({
            "fwd_wgs": int(len(f)),
            "fwd_span_us": round((f[:, 3].max() - t0) / 100.0, 2),
            "fwd_start_spread_us": round((f[:, 0].max() - t0) / 100.0, 2),
            "fwd_rendezvous_med_us": med(f[:, 1] - t0), "fwd_rendezvous_max_us": round((f[:, 1].max() - t0) / 100.0, 2),
            "fwd_loop_entry_med_us": med(f[:, 2] - t0), "fwd_loop_entry_max_us": round((f[:, 2].max() - t0) / 100.0, 2),
            "fwd_end_min_us": round((f[:, 3].min() - t0) / 100.0, 2),
            "bptt_span_us": round((b[b[:, 2] > 0, 1].max() - u0) / 100.0, 2),
            "bptt_rendezvous_med_us": med(rec[:, 6] - u0), "bptt_loop_entry_med_us": med(rec[:, 7] - u0),
            "error_word": int(eng.error_word())}), flush=True)


if __name__ == "__main__":
    main(overrides=sys.argv[1:])
