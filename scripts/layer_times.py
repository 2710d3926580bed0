"""Per-layer kernel times of one steady-state step from a rocprofv3 kernel trace.

A step is the span between the last two post-processing finalize kernels
(k_finalize ends every step); pass a second trace to compare side by side."""
import csv
import sys


def _name(r):
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0].replace('ssa::', '')


def one_step(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if 'k_finalize' in r['Kernel_Name']]
    i0, i1 = (ends[-2] + 1, ends[-1]) if len(ends) >= 2 else (0, len(rows) - 1)
    out = []
    for r in rows[i0:i1 + 1]:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        out.append((_name(r)[:40], d))
    return out


a = one_step(sys.argv[1])
b = one_step(sys.argv[2]) if len(sys.argv) > 2 else None
ta = tb = 0
for i, (n, d) in enumerate(a):
    ta += d
    if b and i < len(b):
        tb += b[i][1]
        print(f"{i:3d} {n:40s} {d:8.1f}  | {b[i][0]:40s} {b[i][1]:8.1f}")
    else:
        print(f"{i:3d} {n:40s} {d:8.1f}")
print("total", round(ta, 1), round(tb, 1))
