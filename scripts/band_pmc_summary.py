"""Per-wave PMC summary of the fused_ir_band kernel over gpurun_out/bpmc* passes."""
import collections
import csv
import glob
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bpmc*"
acc = collections.defaultdict(list)
for d in sorted(p for p in glob.glob(pat) if not p.endswith(".log")):
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if "fused_ir_band" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
waves = sum(acc["SQ_WAVES"]) / max(1, len(acc["SQ_WAVES"]))
for k, v in sorted(acc.items()):
    m = sum(v) / len(v)
    print(f"{k:28s} {m:14.4g}   per wave {m / waves:10.1f}")
