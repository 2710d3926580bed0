#!/bin/bash
# PMC passes over the fused-IR microbench of one block (BLOCK, TILE env)
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
B=${BLOCK:-14}; T=${TILE:-11x11}
timeout -k 10 120 python scripts/bench_fused.py --block $B --tiles $T,5x11 > gpurun_out/fpmc_t.txt 2>&1; cat gpurun_out/fpmc_t.txt
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $REPO/gpurun_out/fpmc$i -o run --output-format csv -- python3 $REPO/scripts/bench_fused.py --block $B --tiles $T --reps 3 > $REPO/gpurun_out/fpmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $REPO/gpurun_out/fpmc$i.log; exit 2; }
done
echo pmc done
