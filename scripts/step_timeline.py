"""Step wall time and GPU busy/overlap from a rocprofv3 kernel trace: per steady-state
step (between consecutive stem kernels), the wall span, the summed kernel time, the
busy union (any kernel running) and the model-only critical path."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
iv = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows]
starts = [s for s, e, n in iv if 'stem_block0' in n or 'stem_conv' in n]
for a, b in zip(starts[-4:-1], starts[-3:]):
    ks = [(s, e, n) for s, e, n in iv if a <= s < b]
    tot = sum(e - s for s, e, _ in ks)
    union, cur_s, cur_e = 0, None, None
    for s, e, _ in sorted(ks):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    model = [(s, e) for s, e, n in ks if not n.lstrip('void ').startswith(('k_', 'ssa::k_', '(anonymous'))]
    print(f"step wall {(b - a) / 1e3:8.1f} us  kernels {tot / 1e3:8.1f}  busy {union / 1e3:8.1f}  "
          f"idle {(b - a - union) / 1e3:6.1f}")
