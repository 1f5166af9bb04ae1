"""What does a side-stream branch cost inside a captured HIP graph on this stack?

Graphs of 12 short spin kernels (torch.cuda._sleep, one workgroup) on the main stream, captured
with and without a side-stream branch forked after kernel 3 and joined before kernel 9 (the shape
of a step whose independent work runs beside a long launch); and the same 12 kernels split into
two graphs replayed back to back (the segment-boundary cost).  Prints per-replay microseconds.
"""
import json

import torch

CYC = int(__import__("os").environ.get("PROBE_CYC", "4000"))   # ~2 us per spin at ~2.1 GHz


def timeit(fn, reps=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


main = torch.cuda.current_stream()
side = torch.cuda.Stream()


def body(branch_cyc=None, lo=0, hi=12):
    for i in range(lo, hi):
        if branch_cyc is not None and i == 3:
            ev = torch.cuda.Event()
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                torch.cuda._sleep(branch_cyc)
            ev2 = torch.cuda.Event()
            ev2.record(side)
        if branch_cyc is not None and i == 9:
            main.wait_event(ev2)
        torch.cuda._sleep(CYC)


def cap(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


out = {}
g0 = cap(lambda: body())
out["serial12_us"] = timeit(g0.replay)
for name, c in (("branch_short", CYC), ("branch_long6", 6 * CYC)):
    g = cap(lambda c=c: body(c))
    out[name + "_us"] = timeit(g.replay)
ga, gb = cap(lambda: body(lo=0, hi=6)), cap(lambda: body(lo=6, hi=12))
out["two_graphs_us"] = timeit(lambda: (ga.replay(), gb.replay()))
one = cap(lambda: torch.cuda._sleep(CYC))
out["one_kernel_graph_us"] = timeit(one.replay)
print(json.dumps({k: round(v, 2) for k, v in out.items()}))
