"""Per-kernel roofline of one learner step from a byte-counter run and a kernel trace.

usage: python tools/roofline.py "gpurun_out/bytes_TAG/p*/**/*counter_collection.csv" \
           gpurun_out/TAG.txt [out.txt]

Inputs: ``tools/gpu.sh bytes TAG`` (FETCH_SIZE / WRITE_SIZE / SQ_VALU_MFMA_BUSY_CYCLES per kernel,
mean over the dispatches of the bench run) and ``tools/gpu.sh prof TAG`` (the step breakdown,
``tools/step_breakdown.py``).  Per kernel:

* MFMA floor = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x 2.4 GHz): the matrix-pipe time of every
  MFMA the kernel issued (32 cycles per 32x32x16 bf16, 16 per 16x16x32 / 16x16x64 i8), spread
  evenly over the chip's SIMDs at the top clock -- the 3-pass split products are counted as what
  they are, three bf16 MFMAs;
* byte floor = (2 x FETCH_SIZE + WRITE_SIZE) / 6.3 TB/s (the measured float4-copy rate; 8 TB/s
  spec).  FETCH_SIZE counts 16-byte-per-lane streaming reads at half their bytes on gfx950
  (MI355X_MICROARCH.md, HBM), so it is doubled; narrower reads are uncalibrated, so the doubled
  figure is an upper bound for kernels that read 4-8 bytes per lane;
* bound = the larger floor; eff = bound / achieved.
"""
import collections
import csv
import glob
import re
import sys

CLK = 2.4e9
SIMDS = 1024
HBM = 6.3e12


def load_counters(pattern):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in sorted(glob.glob(pattern, recursive=True)):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                key = (row["Kernel_Name"], row["Counter_Name"])
                per[key][row.get("Dispatch_Id", "0")] += float(row["Counter_Value"])
    out = collections.defaultdict(dict)
    for (kern, ctr), disp in per.items():
        out[kern][ctr] = sum(disp.values()) / len(disp)
    return out


def load_breakdown(path):
    rows = []
    for ln in open(path):
        m = re.match(r"\s*([\d.]+)us\s+([\d.]+)\s+(.*)$", ln)
        if m:
            rows.append((m.group(3).strip(), float(m.group(1)), float(m.group(2))))
    return rows


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"^_Z\d+", "", name)
    return name.split("(")[0][:44]


def main():
    ctr = load_counters(sys.argv[1])
    rows = load_breakdown(sys.argv[2])
    lines = [f"{'kernel':<44s} {'us':>7s} {'MFMA us':>8s} {'rd MB':>7s} {'wr MB':>7s} {'HBM us':>7s} "
             f"{'bound':>6s} {'eff':>5s}"]
    tot = [0.0, 0.0, 0.0]
    for name, us, _ in rows:
        c = next((v for k, v in ctr.items() if k[:100].startswith(name[:60])), None)
        if c is None:
            lines.append(f"{short(name):<44s} {us:7.1f}   (no counters)")
            continue
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / SIMDS / CLK * 1e6
        rd = 2 * c.get("FETCH_SIZE", 0.0) * 1024 / 1e6
        wr = c.get("WRITE_SIZE", 0.0) * 1024 / 1e6
        hb = (rd + wr) * 1e6 / HBM * 1e6
        floor = max(mf, hb)
        which = "mfma" if mf >= hb else "hbm"
        lines.append(f"{short(name):<44s} {us:7.1f} {mf:8.1f} {rd:7.1f} {wr:7.1f} {hb:7.1f} "
                     f"{which:>6s} {floor / us:5.2f}")
        tot[0] += us
        tot[1] += floor
        tot[2] += mf
    lines.append(f"{'step (sum of kernels)':<44s} {tot[0]:7.1f} {tot[2]:8.1f} {'':>7s} {'':>7s} {'':>7s} "
                 f"{'':>6s} {tot[1] / tot[0]:5.2f}")
    txt = "\n".join(lines)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
