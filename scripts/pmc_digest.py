"""Compact per-kernel digest of the PMC passes (scripts/gpu.sh ... pmc) for one step:
time, MFMA-busy share, wave wait share, LDS bank-conflict share, L2 hit rate,
HBM read/write requests.  python scripts/pmc_digest.py gpurun_out/pmc1 ... pmc4"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    import collections
    import csv

    def load(d):
        disp = collections.OrderedDict()
        for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            e = disp.setdefault(int(r["Dispatch_Id"]), {
                "name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                "t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
            e[r["Counter_Name"]] = float(r["Counter_Value"])
        ds = list(disp.values())
        idx = [i for i, d in enumerate(ds) if "k_finalize" in d["name"]]
        return ds[idx[-2] + 1: idx[-1] + 1]

    steps = [load(d) for d in sys.argv[1:]]
    n = min(len(s) for s in steps)
    print(f"{'kernel':34s} {'t_us':>7s} {'mfma%':>6s} {'wait%':>6s} {'ldsI/w':>7s} {'bank%':>6s} "
          f"{'L2hit%':>6s} {'rdMB':>7s} {'wrMB':>7s}")
    for i in range(n):
        d = {}
        for s in steps:
            d.update(s[i])
        nm = d["name"].split("(")[0].replace("void ", "").replace("ssa::", "").replace(
            "(anonymous namespace)::", "")[:34]
        gui = d.get("GRBM_GUI_ACTIVE", 0) or 1
        mfma = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui * 256 * 4) * 100
        wait = d.get("SQ_WAIT_ANY", 0) / max(1, d.get("SQ_WAVE_CYCLES", 1)) * 100
        ldsi = d.get("SQ_INSTS_LDS", 0) / max(1, d.get("SQ_WAVES", 1))
        bank = d.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, d.get("SQ_ACTIVE_INST_LDS", 1)) * 100
        h, m = d.get("TCC_HIT_sum", 0), d.get("TCC_MISS_sum", 0)
        hit = h / max(1, h + m) * 100
        rd = d.get("TCC_EA0_RDREQ_sum", 0) * 64 / 1e6
        wr = d.get("TCC_EA0_WRREQ_sum", 0) * 64 / 1e6
        print(f"{nm:34s} {d['t']:7.1f} {mfma:6.1f} {wait:6.1f} {ldsi:7.0f} {bank:6.1f} {hit:6.1f} "
              f"{rd:7.1f} {wr:7.1f}")


if __name__ == "__main__":
    main()
