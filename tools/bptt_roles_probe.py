"""Per-role clock stamps of the fp32 BPTT launch (lstm_persist.hip lstm_bwd_tag_kernel, PTBArgs::dbg)
at the bench config, one eager engine step per arm, arms as learner.* override sets:

    python tools/bptt_roles_probe.py hoist=0 off hoist_stop_lead=3 ...

Per arm: launch span (first workgroup start -> last workgroup end), the recurrence's end (its
last workgroup), the helpers' end (head-gradient reduction), the median / max BPTT iteration of
recurrence workgroup (0, 0) and the medians of its first / middle / last 10 iterations (round 6:
in the hoisted step the side branch's priority tail + sample run beside the first ~15
iterations, its torso frames beside the rest).  Times in us (s_memrealtime, 100 MHz, one clock
for the chip).
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


def arm(spec: str, reps: int = 3):
    over = {"seed": 1234, "learner.use_graph": False}
    for kv in filter(None, spec.split(",")):
        if kv == "off":
            continue
        key, _, val = kv.partition("=")
        over["learner." + key] = val
    cfg = get_config("atari57", **over)
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
    out = []
    for _ in range(reps):
        dbg = torch.zeros(4096, dtype=torch.int64, device=DEV)
        k.r2_lstm_persist_set_debug(ptr(dbg))
        eng.step()
        torch.cuda.synchronize()
        k.r2_lstm_persist_set_debug(None)
        d = dbg.cpu().numpy()
        blk = d[:2048].reshape(256, 8)
        rec, hlp = blk[blk[:, 2] == 1], blk[blk[:, 2] == 2]
        # the forward launch shares the debug pointer (its words 256+ / per-step stamps): only the
        # BPTT writes role words, so select by role
        t0 = int(blk[blk[:, 2] > 0, 0].min())
        us = lambda x: round(float(x) / 100.0, 2)   # noqa: E731  (10 ns ticks)
        it = d[2048:2048 + 40]
        it = it[it > 0]
        dit = np.diff(it) / 100.0
        # recurrence workgroup (0, 0) is the one stamping iterations: find it as the recurrence
        # block whose start is closest before the first iteration stamp
        rec_start = rec[:, 0]
        w00 = rec_start[rec_start <= it[0]].max() if len(it) and (rec_start <= it[0]).any() else rec_start.min()
        r = {"span_us": us(blk[blk[:, 2] > 0, 1].max() - t0),
             "startup_us": us(it[0] - t0) if len(it) else None,
             "first_iter_us": us(it[1] - it[0]) if len(it) > 1 else None,
             "after_last_iter_us": us(rec[:, 1].max() - it[-1]) if len(it) else None,
             "wg00_start_us": us(w00 - t0),
             "recurrence_end_us": us(rec[:, 1].max() - t0),
             "recurrence_start_spread_us": us(rec[:, 0].max() - rec[:, 0].min()),
             # per recurrence workgroup: start -> XCD rendezvous done -> loop entry (medians)
             "rendezvous_med_us": us(np.median(rec[:, 6] - rec[:, 0])),
             "rendezvous_max_us": us((rec[:, 6] - rec[:, 0]).max()),
             "loop_entry_med_us": us(np.median(rec[:, 7] - rec[:, 0])),
             "loop_entry_max_us": us((rec[:, 7] - rec[:, 0]).max()),
             "iter_med_us": round(float(np.median(dit)), 3) if len(dit) else None,
             "iter_max_us": round(float(dit.max()), 3) if len(dit) else None,
             "iter_med_first10": round(float(np.median(dit[:10])), 3) if len(dit) >= 30 else None,
             "iter_med_mid10": round(float(np.median(dit[10:20])), 3) if len(dit) >= 30 else None,
             "iter_med_last10": round(float(np.median(dit[-10:])), 3) if len(dit) >= 30 else None,
             "n_helpers": int(len(hlp))}
        if len(hlp):
            r.update({"helpers_end_us": us(hlp[:, 1].max() - t0),
                      "helpers_end_med_us": us(np.median(hlp[:, 1]) - t0)})
        out.append(r)
    err = eng.error_word()
    return {"arm": spec, "error_word": int(err), "runs": out}


def main():
    arms = sys.argv[1:] or ["hoist=0", "off"]
    for a in arms:
        print(json.dumps(arm(a)), flush=True)


if __name__ == "__main__":
    main()
