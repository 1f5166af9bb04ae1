"""Median duration (us) per kernel name over the timed steps of a rocprofv3 kernel trace.

    python tools/kernel_medians.py 'gpurun_out/prof_TAG/*/*kernel_trace.csv' [name filters...]
"""
import csv
import glob
import statistics
import sys


def main(pattern, filters):
    rows = list(csv.DictReader(open(sorted(glob.glob(pattern))[-1])))
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"][:48], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(by.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
        if filters and not any(f in k for f in filters):
            continue
        tail = v[len(v) // 2:]            # the later half: graph replays, not the eager warm-up
        print("%-48s n=%4d med %8.1f  med(late half) %8.1f" % (k, len(v), statistics.median(v),
                                                                statistics.median(tail)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
