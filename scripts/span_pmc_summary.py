"""Average PMC counters per kernel name over the span microbenchmark passes:
python scripts/span_pmc_summary.py gpurun_out/spmc1 gpurun_out/spmc2 ..."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[-60:]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[name]["_vgpr"].append(float(r["VGPR_Count"]))
        acc[name]["_lds"].append(float(r["LDS_Block_Size"]))
for name, cs in acc.items():
    print(name)
    for k in sorted(cs):
        v = cs[k]
        print(f"   {k:28s} {sum(v) / len(v):14.4g}   (n={len(v)})")
