"""Per-kernel times of one steady-state step from a rocprofv3 kernel trace.

Every kernel of the step is listed once per launch slot, in launch order, with its
duration averaged over the traced steps after the first two (warm-up). A step ends with
the post-processing's last kernel (k_finalize; k_records since the round-3 merge).
Round 1-3 versions took the span between the last two step ends, which drops the model
kernels of the next step that the post-processing stream interleaves with.
Pass a second trace to compare side by side."""
import csv
import sys


def _name(r):
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0].replace('ssa::', '')


def one_step(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if 'k_finalize' in r['Kernel_Name'] or 'k_records' in r['Kernel_Name']]
    if len(ends) < 4:
        i0, i1 = (ends[-2] + 1, ends[-1]) if len(ends) >= 2 else (0, len(rows) - 1)
        return [(_name(r)[:40], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
                for r in rows[i0:i1 + 1]]
    # steady steps: between the 2nd and the last step end; the kernels of each name are
    # launched the same number of times per step, so the k-th launch of a name in a step is
    # slot (name, k); slots are ordered by their first appearance
    body = rows[ends[1] + 1:ends[-1] + 1]
    nsteps = len(ends) - 2
    seq, order, count = {}, [], {}
    for r in body:
        n = _name(r)[:40]
        count[n] = count.get(n, 0) + 1
    per_step = {n: c // nsteps for n, c in count.items() if c >= nsteps}
    seen = {}
    for r in body:
        n = _name(r)[:40]
        if n not in per_step:
            continue
        k = seen.get(n, 0) % per_step[n]
        seen[n] = seen.get(n, 0) + 1
        key = (n, k)
        if key not in seq:
            seq[key] = []
            order.append(key)
        seq[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    return [(n, sum(v) / len(v)) for (n, k), v in ((key, seq[key]) for key in order)]


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
