"""Do independent branches of a captured HIP graph run concurrently on this stack?

Two spin kernels (torch.cuda._sleep, one workgroup each) on two streams, eager and captured
with a fork/join; prints the replay time relative to one kernel.  ~1.0 = concurrent, ~2.0 =
serialised.
"""
import json

import torch


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


CYC = 2_000_000
s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
one = timeit(lambda: torch.cuda._sleep(CYC))


def two():
    ev = torch.cuda.Event()
    ev.record(s0)
    s1.wait_event(ev)
    torch.cuda._sleep(CYC)
    with torch.cuda.stream(s1):
        torch.cuda._sleep(CYC)
    ev2 = torch.cuda.Event()
    ev2.record(s1)
    s0.wait_event(ev2)


eager = timeit(two)
g = torch.cuda.CUDAGraph()
two()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    two()
graph = timeit(g.replay)
print(json.dumps({"one_us": round(one, 1), "eager_two_streams_ratio": round(eager / one, 2),
                  "graph_two_branches_ratio": round(graph / one, 2)}))
