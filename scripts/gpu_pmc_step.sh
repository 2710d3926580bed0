#!/bin/bash
# PMC passes over a short headline bench (sequential model): per-kernel SQ counters
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
O=gpurun_out/pmc_step
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH"; do
  i=$((i+1))
  SSA_SLOT_PARALLEL=0 timeout -s KILL 180 rocprofv3 --pmc $set -d $REPO/$O/p$i -o run --output-format csv -- python3 $REPO/bench.py --steps 3 --warmup 1 --lag 1 --rpc 0 > $REPO/$O/p$i.log 2>&1 || { echo "set $i failed rc=$?"; tail -5 $REPO/$O/p$i.log; exit 1; }
done
cd $REPO
python3 scripts/pmc_summary.py $O/p1 $O/p2 $O/p3 > $O/summary.txt 2>&1 || true
head -60 $O/summary.txt
