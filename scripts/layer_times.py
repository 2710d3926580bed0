"""Per-layer kernel times of one graph replay from a rocprofv3 kernel trace."""
import csv
import sys


def one_step(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if 'stem_kernel' in r['Kernel_Name']]
    i0 = idx[-1]
    out = []
    for r in rows[i0:]:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('ssa::', '').replace('(anonymous namespace)::', '')
        out.append((n[:34], d))
        if 'k_finalize' in r['Kernel_Name']:
            break
    return out


a = one_step(sys.argv[1])
b = one_step(sys.argv[2]) if len(sys.argv) > 2 else None
ta = tb = 0
for i, (n, d) in enumerate(a):
    ta += d
    if b and i < len(b):
        tb += b[i][1]
        print(f"{i:3d} {n:34s} {d:8.1f}  | {b[i][0]:34s} {b[i][1]:8.1f}")
    else:
        print(f"{i:3d} {n:34s} {d:8.1f}")
print("total", round(ta, 1), round(tb, 1))
