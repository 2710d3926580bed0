#!/bin/bash
# PMC passes over the fused_ir_band microbenchmark: BLOCK=1 R=7 NSLOT=1
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 120 python scripts/bench_band.py --block ${BLOCK:-1} --R ${R:-7} --nslot ${NSLOT:-1} || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $REPO/gpurun_out/bpmc$i -o run --output-format csv -- python3 $REPO/scripts/bench_band.py --block ${BLOCK:-1} --R ${R:-7} --nslot ${NSLOT:-1} --reps 3 > $REPO/gpurun_out/bpmc$i.log 2>&1 || { echo "set $i failed rc=$?"; tail -5 $REPO/gpurun_out/bpmc$i.log; exit 1; }
done
echo done
