"""Per-kernel PMC ratios of one B=32 step from scripts/gpu.sh's 3 pmc passes:
python scripts/pmc_step.py DIR  (DIR/pmc1..3). Aligns the passes at the second-to-last
stem_band dispatch (the sequential trace's steady step) and prints, per kernel, LDS bank
conflict cycles per LDS instruction, the waiting share of wave cycles and the kernel time."""
import sys

exec(open(__file__.replace("pmc_step.py", "pmc_summary.py")).read()
     .split("steps = [last_step(s) for s in sets]")[0]
     .replace("sets = [load(d) for d in sys.argv[1:]]",
              "sets = [load(f'{sys.argv[1]}/pmc{i}') for i in (1, 2, 3)]"))


def window(ds, n=40):
    idx = [i for i, d in enumerate(ds) if "stem_band_kernel" in d["name"]]
    return ds[idx[-2]:idx[-2] + n]


ws = [window(s) for s in sets]
for i in range(min(len(w) for w in ws)):
    names = {w[i]["name"].split("(")[0] for w in ws}
    d = {}
    for w in ws:
        d.update(w[i])
    nm = d["name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("ssa::", "")[:44]
    lds = d.get("SQ_INSTS_LDS", 0)
    flag = "" if len(names) == 1 else "  (passes misaligned)"
    print(f"{nm:44s} conflicts/LDS-instr {d.get('SQ_LDS_BANK_CONFLICT', 0) / max(lds, 1):5.2f}  "
          f"wait {d.get('SQ_WAIT_ANY', 0) / max(d.get('SQ_WAVE_CYCLES', 1), 1):4.2f}  "
          f"LDS-instr/wave {lds / max(d.get('SQ_WAVES', 1), 1):6.0f}  t {d['t']:6.1f} us{flag}")
    if "k_records" in nm:
        break
