"""One line per kernel from a pmc_kernels.py report (scripts/gpu.sh pmck -> kernel_pmc.txt):
time per dispatch, waves, instructions per wave by class, MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES
per GRBM_GUI_ACTIVE cycle and SIMD, x 100 / 16 CUs' share as in the round-6 tables) and LDS
bank-conflict cycles per LDS instruction. Our HIP kernels only (vendor / runtime kernels
skipped), sorted by time per dispatch.

  python scripts/pmc_kernel_table.py gpurun_out/<dir>/kernel_pmc.txt
"""
import re
import sys


def main():
    blocks, cur = [], None
    for line in open(sys.argv[1]):
        m = re.match(r"== (.*?) grid=(\d+) vgpr=(\S+)\s+\(~([\d.]+) us/dispatch\)", line)
        if m:
            cur = dict(name=m.group(1), grid=int(m.group(2)), vgpr=m.group(3), us=float(m.group(4)), c={})
            blocks.append(cur)
            continue
        m = re.match(r"\s+([A-Z_]+)\s+(\d+)", line)
        if m and cur is not None:
            cur["c"][m.group(1)] = int(m.group(2))
    skip = ("__amd", "at::", "Tensor", "elementwise", "Im2", "kernelHistogram", "Cijk", "void at", "naive_",
            "_ZN2ck", "miopen", "Sub", "MIOpen", "gemm", "batched", "igemm")  # startup fp32 reference / vendor kernels
    print(f"# {'kernel':44s} {'grid':>9s} {'vgpr':>7s} {'us':>7s} {'waves':>7s} {'MFMA/w':>7s} {'VALU/w':>7s} "
          f"{'SALU/w':>7s} {'LDS/w':>6s} {'VMRD/w':>6s} {'mfmaB':>6s} {'ldsCf':>6s}")
    for b in sorted(blocks, key=lambda b: -b["us"]):
        if b["name"].startswith(skip) or not b["c"].get("SQ_WAVES"):
            continue
        c, w = b["c"], b["c"]["SQ_WAVES"]
        pw = lambda k: c.get(k, 0) / w
        gui = c.get("GRBM_GUI_ACTIVE", 0)
        mfmab = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / gui / 1024 * 16 / 4 if gui else 0.0
        lds = c.get("SQ_INSTS_LDS", 0)
        cf = c.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else 0.0
        print(f"{b['name'][:46]:46s} {b['grid']:9d} {b['vgpr']:>7s} {b['us']:7.1f} {w:7d} {pw('SQ_INSTS_MFMA'):7.0f} "
              f"{pw('SQ_INSTS_VALU'):7.0f} {pw('SQ_INSTS_SALU'):7.0f} {pw('SQ_INSTS_LDS'):6.0f} {pw('SQ_INSTS_VMEM_RD'):6.0f} "
              f"{mfmab:6.2f} {cf:6.2f}")


if __name__ == "__main__":
    main()
