"""Per-step timeline of the hoisted learner step from a rocprofv3 kernel trace: each kernel's
start / end relative to the step's first main-stream torso launch (us), queue id, duration.

    python tools/hoist_timeline.py 'gpurun_out/prof_TAG/*/*kernel_trace.csv' [step index]
"""
import csv
import glob
import sys


def main(pattern, which=-2):
    rows = list(csv.DictReader(open(sorted(glob.glob(pattern))[-1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    S = lambda r: int(r["Start_Timestamp"])   # noqa: E731
    E = lambda r: int(r["End_Timestamp"])     # noqa: E731
    # the step's main torso launch: the torso launch followed on its queue by the x-projection
    def main_torso(i):
        r = rows[i]
        if "torso_fwd_sp2" not in r["Kernel_Name"]:
            return False
        nxt = next((o for o in rows[i + 1:] if o["Queue_Id"] == r["Queue_Id"]), None)
        return nxt is not None and "gemm6_kernel<true, 192, 256" in nxt["Kernel_Name"]
    starts = [i for i in range(len(rows)) if main_torso(i)]
    i0, i1 = starts[which], starts[which + 1] if which + 1 < len(starts) else len(rows)
    t0 = S(rows[i0])
    print("%-44s %5s %9s %9s %8s" % ("kernel", "queue", "start", "end", "us"))
    for r in rows[i0:i1]:
        print("%-44s %5s %9.1f %9.1f %8.1f" % (r["Kernel_Name"][:44], r["Queue_Id"], (S(r) - t0) / 1e3,
                                             (E(r) - t0) / 1e3, (E(r) - S(r)) / 1e3))
    print("step span (torso start -> next torso start): %.1f us" % ((S(rows[i1]) - t0) / 1e3 if i1 < len(rows) else 0))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else -2)
