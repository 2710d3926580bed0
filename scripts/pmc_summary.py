"""Per-kernel PMC summary of the last bench step: python scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 ..."""
import collections
import csv
import sys


def load(d):
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    # group by dispatch
    disp = collections.OrderedDict()
    for r in rows:
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                "lds": int(r["LDS_Block_Size"]), "vgpr": int(r["VGPR_Count"]),
                                "agpr": int(r["Accum_VGPR_Count"]),
                                "t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    return list(disp.values())


sets = [load(d) for d in sys.argv[1:]]
# last step: from the last stem_kernel dispatch on
def last_step(ds):
    # one steady-state step: after the second-to-last post-processing finalize
    idx = [i for i, d in enumerate(ds) if "k_finalize" in d["name"] or "k_records" in d["name"]]
    return ds[idx[-2] + 1: idx[-1] + 1] if len(idx) >= 2 else ds


steps = [last_step(s) for s in sets]
n = min(len(s) for s in steps)
keys = []
for s in steps:
    for k in s[0]:
        if k.isupper() or k.startswith("SQ") or k.startswith("GRBM"):
            if k not in keys:
                keys.append(k)
print("idx name                              grid   lds  vgpr/agpr " + " ".join(f"{k[:14]:>14s}" for k in keys))
for i in range(n):
    d = {}
    for s in steps:
        d.update({k: v for k, v in s[i].items()})
    nm = d["name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("ssa::", "")[:32]
    print(f"{i:3d} {nm:32s} {d['grid']:7d} {d['lds']:6d} {d['vgpr']:3d}/{d['agpr']:<3d} " +
          " ".join(f"{d.get(k, float('nan')):14.4g}" for k in keys))
