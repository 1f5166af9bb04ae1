"""Overlap of two roles' kernels in a rocprofv3 kernel trace (concurrent actor / learner).

Kernels are attributed to a role by queue id (each CU-masked stream gets its own HW queue); the
steady-state window is the last ``--frac`` of the trace.  Reports each queue's busy time, the
union, and the time both queues were busy at once.

    python tools/trace_overlap.py gpurun_out/prof_conc/conc_kernel_trace.csv
"""
import argparse
import collections
import csv


def merge(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(iv):
    return sum(b - a for a, b in iv)


def intersect(x, y):
    i = j = 0
    out = []
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append([a, b])
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--frac", type=float, default=0.5)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    lo = t1 - (t1 - t0) * a.frac
    by_q = collections.defaultdict(list)
    names = collections.defaultdict(collections.Counter)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < lo:
            continue
        q = r["Queue_Id"]
        by_q[q].append((s, e))
        names[q][r["Kernel_Name"].split("(")[0][:48]] += 1
    win = t1 - lo
    print(f"window {win / 1e6:.2f} ms")
    merged = {q: merge(v) for q, v in by_q.items()}
    for q, iv in sorted(merged.items(), key=lambda kv: -length(kv[1])):
        top = ", ".join(f"{n} x{c}" for n, c in names[q].most_common(3))
        print(f"queue {q}: {len(by_q[q])} kernels, busy {length(iv) / 1e6:.2f} ms "
              f"({100 * length(iv) / win:.0f}%)  [{top}]")
    qs = sorted(merged, key=lambda q: -length(merged[q]))
    if len(qs) >= 2:
        x, y = merged[qs[0]], merged[qs[1]]
        both = intersect(x, y)
        union = merge(x + y)
        print(f"union busy {length(union) / 1e6:.2f} ms ({100 * length(union) / win:.0f}%), "
              f"both busy {length(both) / 1e6:.2f} ms ({100 * length(both) / max(1, length(y)):.0f}% "
              f"of queue {qs[1]})")


if __name__ == "__main__":
    main()
