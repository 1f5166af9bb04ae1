"""Per-kernel timeline of the last steady-state learner step in a rocprofv3 kernel trace:
start offset, duration, idle gap before it (us)."""
import csv
import glob
import os
import sys


def main(path_glob, marker="step_end"):
    p = sorted(glob.glob(path_glob), key=os.path.getmtime)[-1]
    rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    st = rows[ends[-2] + 1: ends[-1] + 1]
    t0 = int(st[0]["Start_Timestamp"])
    prev = t0
    busy = 0
    for r in st:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {(s - prev) / 1e3:6.1f}  {r['Kernel_Name'][:60]}")
        busy += e - s
        prev = max(prev, e)
    print(f"wall {(prev - t0) / 1e3:.1f} us, kernel-busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
