"""Per-kernel-name PMC means over every dispatch of rocprofv3 --pmc runs (one dir per
counter set): python scripts/pmc_kernels.py DIR [DIR ...]. Used for standalone harnesses
(csrc/tools/post_bench.hip) where every dispatch is a kernel of interest."""
import collections
import csv
import glob
import os
import sys

BY_GRID = os.environ.get("PMC_BY_GRID") == "1"  # key by kernel name + grid size (one layer per key)


def load(d):
    f = (glob.glob(f"{d}/*/run_counter_collection.csv") + glob.glob(f"{d}/run_counter_collection.csv"))[0]
    disp = {}
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        name = (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                .replace("void ", "").replace("ssa::", ""))
        if BY_GRID:
            name += f" grid={r.get('Grid_Size', '?')} vgpr={r.get('VGPR_Count', '?')}/{r.get('Accum_VGPR_Count', '?')}"
        e = disp.setdefault(k, {"name": name, "t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(disp.values())


agg = collections.OrderedDict()
for d in sys.argv[1:]:
    for e in load(d):
        a = agg.setdefault(e["name"], collections.defaultdict(list))
        for k, v in e.items():
            if k != "name":
                a[k].append(v)
for name, a in agg.items():
    m = {k: sum(v) / len(v) for k, v in a.items()}
    waves = m.get("SQ_WAVES", 0) or 1
    print(f"== {name}  (~{m['t']:.1f} us/dispatch)")
    for k in sorted(m):
        if k == "t":
            continue
        extra = f"   per wave {m[k] / waves:10.1f}" if k.startswith("SQ_INSTS") or k.startswith("SQ_WAIT") else ""
        print(f"   {k:28s} {m[k]:14.0f}{extra}")
