"""Same-process A/B of the fp32 torso forward between kernel-library builds: each library is loaded
with its own ctypes handle (its own code objects), the same frames / weights / jobs run through
r2_torso_fwd_sp_multi of each, interleaved over rounds (min of the per-round means), plus the
per-phase clock stamps of workgroup 0 (median cycles per frame and wave).

    python tools/torso_lib_ab.py name=path/to/_r2d2_kernels.so ... [--bits N,...]
"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

DEV = torch.device("cuda")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def main():
    libs, bits = [], [0]
    for a in sys.argv[1:]:
        if a.startswith("--bits"):
            bits = [int(v) for v in a.split("=", 1)[1].split(",")]
        else:
            name, _, path = a.partition("=")
            lib = ctypes.CDLL(os.path.abspath(path))
            for fn in ("r2_torso_fwd_sp_multi", "r2_torso_sp_trace", "r2_torso_sp_debug"):
                getattr(lib, fn).restype = ctypes.c_int
            lib.r2_torso_fwd_sp_multi.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                  ctypes.c_int, ctypes.c_void_p]
            lib.r2_torso_sp_trace.argtypes = [ctypes.c_void_p]
            lib.r2_torso_sp_debug.argtypes = [ctypes.c_int]
            libs.append((name, lib))
    g = torch.Generator(device=DEV).manual_seed(0)
    B, T, n, Lb, cap = 64, 80, 5, 40, 200_000
    frames = torch.randint(0, 256, (cap, 4 * 84 * 84), dtype=torch.uint8, device=DEV, generator=g)
    rows = torch.randint(0, cap, ((T + n) * B,), dtype=torch.int32, device=DEV, generator=g)

    def split(x):
        hi = x.to(torch.bfloat16)
        return hi, (x - hi.float()).to(torch.bfloat16)

    def net():
        w = [split(torch.randn(32, k, device=DEV, generator=g) * 0.05) for k in (256, 512, 288)]
        b = [torch.randn(32, device=DEV, generator=g) * 0.1 for _ in range(3)]
        return w, b

    (on_w, on_b), (tg_w, tg_b) = net(), net()
    Xo = torch.empty(2, (T + n) * B, 1568, dtype=torch.bfloat16, device=DEV)
    Xt = torch.empty(2, T * B, 1568, dtype=torch.bfloat16, device=DEV)
    NL = (T - Lb) * B
    s1 = torch.empty(2, NL, 400, 32, dtype=torch.bfloat16, device=DEV)
    s2 = torch.empty(2, NL, 81, 32, dtype=torch.bfloat16, device=DEV)
    p = lambda t: t.data_ptr()   # noqa: E731

    def job(w, b, r, X, save):
        return [p(r), r.numel(), p(w[0][0]), p(w[0][1]), p(b[0]), p(w[1][0]), p(w[1][1]), p(b[1]),
                p(w[2][0]), p(w[2][1]), p(b[2]), p(X[0]), p(X[1]), p(s1[0]) if save else 0,
                p(s1[1]) if save else 0, p(s2[0]) if save else 0, p(s2[1]) if save else 0, 0, 0, 0]

    jobs = np.asarray([job(on_w, on_b, rows[: Lb * B], Xo[:, : Lb * B], False),
                       job(on_w, on_b, rows[Lb * B: T * B], Xo[:, Lb * B: T * B], True),
                       job(on_w, on_b, rows[T * B:], Xo[:, T * B:], False),
                       job(tg_w, tg_b, rows[n * B:], Xt, False)], dtype=np.int64)
    n_cus = torch.cuda.get_device_properties(0).multi_processor_count
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run(lib):
        rc = lib.r2_torso_fwd_sp_multi(ctypes.c_void_p(frames.data_ptr()),
                                       ctypes.c_void_p(jobs.ctypes.data), 4, n_cus, stream)
        assert rc == 0, rc

    def timeit(lib, reps=10):
        run(lib)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run(lib)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1000.0

    out = {}
    for _ in range(7):
        for name, lib in libs:
            for b in bits:
                lib.r2_torso_sp_debug(b)
                k = f"{name}_bits{b}_us"
                out[k] = round(min(out.get(k, 1e30), timeit(lib)), 1)
                lib.r2_torso_sp_debug(0)
    for name, lib in libs:
        tr = torch.zeros(8 * 16 * 5, dtype=torch.int64, device=DEV)
        lib.r2_torso_sp_trace(ctypes.c_void_p(tr.data_ptr()))
        run(lib)
        torch.cuda.synchronize()
        lib.r2_torso_sp_trace(None)
        t = tr.view(8, 16, 5).cpu().tolist()
        out[f"{name}_phaseA_med_cycles"] = [int(statistics.median(f[1] - f[0] for f in t[w][2:12])) for w in range(8)]
        out[f"{name}_phaseB_med_cycles"] = [int(statistics.median(f[3] - f[2] for f in t[w][2:12])) for w in range(8)]
        out[f"{name}_frame_med_cycles"] = int(statistics.median(t[0][i + 1][0] - t[0][i][0] for i in range(2, 12)))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
