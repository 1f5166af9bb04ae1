"""Summarise one steady-state learner step from a rocprofv3 --kernel-trace CSV."""
import collections
import csv
import glob
import sys


def main(path_glob, out=None, last=1, marker=('step_end', 'prio_tail', 'tree_update_tail')):
    import os
    paths = sorted(glob.glob(path_glob), key=os.path.getmtime, reverse=True)
    rows = list(csv.DictReader(open(paths[0])))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = (marker,) if isinstance(marker, str) else marker
    # the first marker present in the trace ends a step (step_end_kernel when the tree repair
    # runs on the side stream, the fused tree tail otherwise)
    marks = [m for m in marks if any(m in r['Kernel_Name'] for r in rows)][:1]
    ends = [i for i, r in enumerate(rows) if any(m in r['Kernel_Name'] for m in marks)]
    a, b = ends[-1 - last] + 1, ends[-1] + 1
    st = rows[a:b]
    t0 = int(st[0]['Start_Timestamp'])
    t1 = int(st[-1]['End_Timestamp'])
    lines = [f"steps {last}  wall/step us {(t1 - t0) / 1e3 / last:.1f}  kernels/step {len(st) / last:.0f}"]
    agg = collections.OrderedDict()
    for r in st:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 / last
        c = agg.setdefault(r['Kernel_Name'][:110], [0, 0.0])
        c[0] += 1
        c[1] += d
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
        lines.append(f"{d:9.1f}us {c / last:6.1f}  {n}")
    txt = "\n".join(lines)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None,
         int(sys.argv[3]) if len(sys.argv) > 3 else 1,
         sys.argv[4] if len(sys.argv) > 4 else ('step_end', 'prio_tail', 'tree_update_tail'))
