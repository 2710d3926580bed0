"""Per-kernel EXCLUSIVE time in a concurrent (slot-parallel) kernel trace: the time a
kernel runs with no other kernel in flight. In the concurrent regime those intervals
are what sets the step time; kernels that always overlap cost little extra.

  python scripts/exclusive_time.py run_kernel_trace.csv [skip_first_ms]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
if skip < 0:  # negative: keep only the last |skip| ms of the trace
    t_end = max(int(r["End_Timestamp"]) for r in rows)
    rows = [r for r in rows if (t_end - int(r["Start_Timestamp"])) / 1e6 <= -skip]
    skip = 0.0


def name(r):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].replace("ssa::", "")[:44]


ev = []
t_first = min(int(r["Start_Timestamp"]) for r in rows)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if (s - t_first) / 1e6 < skip:
        continue
    ev.append((s, 1, name(r)))
    ev.append((e, -1, name(r)))
ev.sort()
active = collections.Counter()
excl = collections.Counter()
busy = idle = 0.0
total = collections.Counter()
last = ev[0][0]
for t, d, n in ev:
    dt = (t - last) / 1e3
    live = [k for k, v in active.items() if v > 0]
    if len(live) == 1:
        excl[live[0]] += dt
    if live:
        busy += dt
    else:
        idle += dt
    last = t
    active[n] += d
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if (s - t_first) / 1e6 >= skip:
        total[name(r)] += (e - s) / 1e3
span = (ev[-1][0] - ev[0][0]) / 1e3
print(f"span {span:.1f} us, busy {busy:.1f}, idle {idle:.1f}; kernel-time sum {sum(total.values()):.1f}")
print(f"{'kernel':46s} {'sum us':>10s} {'exclusive':>10s}")
for n, v in sorted(total.items(), key=lambda kv: -excl[kv[0]])[:30]:
    print(f"{n:46s} {v:10.1f} {excl[n]:10.1f}")
