"""GPU busy fraction and kernel concurrency of a slot-parallel bench run, from a
rocprofv3 kernel trace (``--kernel-trace``, csv): over the last ``count`` steps of the run
(from the start of the count-th last ``marker`` kernel -- one per step, default the
post-processing's ``k_records`` -- to the end of the last one: the timed steps, start-up,
plan build and autotune excluded), the share of wall time with at least one kernel
executing, the mean number of kernels executing, and the time-weighted share of each
kernel family. Answers whether the step is bound by kernel work (busy ~1) or by gaps
(launch, host, event waits).

  python scripts/busy_fraction.py run_kernel_trace.csv [marker] [count]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_records"
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    ks = []
    for r in csv.DictReader(open(path)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    marks = [k for k in ks if marker in k[2]]
    if len(marks) < count + 1:
        raise SystemExit(f"only {len(marks)} {marker} kernels in the trace")
    a, b = marks[-count - 1][1], marks[-1][1]  # count whole steps: end of one marker to the last
    ev = []
    fam = defaultdict(float)
    for s, e, n in ks:
        s, e = max(s, a), min(e, b)
        if e <= s:
            continue
        ev.append((s, 1))
        ev.append((e, -1))
        fam[n.split("<")[0].split("(")[0][:40]] += (e - s)
    ev.sort()
    busy = conc = 0.0
    cur, last = 0, a
    for t, d in ev:
        if cur > 0:
            busy += t - last
            conc += cur * (t - last)
        cur += d
        last = t
    span = b - a
    print(f"last {count} steps ({marker}): window {span / 1e3:.1f} us, {span / count / 1e3:.1f} us per step: busy {busy / span:.3f}, mean kernels in flight "
          f"{conc / span:.2f} (while busy {conc / max(busy, 1):.2f})")
    tot = sum(fam.values())
    for n, v in sorted(fam.items(), key=lambda x: -x[1])[:20]:
        print(f"  {n:40s} {v / tot:6.3f}")


if __name__ == "__main__":
    main()
