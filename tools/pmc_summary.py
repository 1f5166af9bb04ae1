"""Summarise rocprofv3 --pmc passes (tools/pmc_torso.sh, tools/pmc_gemm.sh) into one text table.

usage: python tools/pmc_summary.py "gpurun_out/pmc/p*/**/*counter_collection.csv" [kernel-substring ...]

Per kernel and counter: the mean over dispatches of the dispatch's value (rows of one dispatch,
e.g. per-XCC dimensions, are summed first).  Derived ratios are printed when their counters exist.
"""
import collections
import csv
import glob
import sys


def load(pattern):
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, ctr) -> {disp: v}
    for path in sorted(glob.glob(pattern, recursive=True)):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                key = (row["Kernel_Name"], row["Counter_Name"])
                per[key][row.get("Dispatch_Id", row.get("Correlation_Id", "0"))] += float(row["Counter_Value"])
    out = collections.defaultdict(dict)
    for (kern, ctr), disp in per.items():
        out[kern][ctr] = sum(disp.values()) / len(disp)
    return out


def ratio(c, a, b):
    return c[a] / c[b] if a in c and b in c and c[b] else None


def main():
    pattern = sys.argv[1]
    wanted = sys.argv[2:]
    data = load(pattern)
    for kern in sorted(data):
        if wanted and not any(w in kern for w in wanted):
            continue
        c = data[kern]
        print(kern[:100])
        for ctr in sorted(c):
            print(f"   {ctr:<30s} {c[ctr]:>12.4g}")
        derived = [("wait_any/wave_cycles", ratio(c, "SQ_WAIT_ANY", "SQ_WAVE_CYCLES")),
                   ("lds_bank_conflict/lds_active", ratio(c, "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE")),
                   ("valu/mfma", ratio(c, "SQ_INSTS_VALU", "SQ_INSTS_VALU_MFMA_BF16")),
                   ("mfma_busy/busy_cycles", ratio(c, "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES"))]
        txt = "; ".join(f"{n} = {v:.2f}" for n, v in derived if v is not None)
        if txt:
            print("   " + txt)


if __name__ == "__main__":
    main()
