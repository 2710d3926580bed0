#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 per counter set; no trace modes).
# The plan is tuned once (SSA_TUNE_FILE) so every pass runs the same kernels.
# Summary: python scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1 SSA_TUNE_FILE=$REPO/gpurun_out/pmc_tune.json
rm -f $SSA_TUNE_FILE
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --rpc 0 ${BENCH_ARGS:-} > gpurun_out/pmc_tune.log 2>&1 || { tail -5 gpurun_out/pmc_tune.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_CVT FETCH_SIZE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  echo "== pmc set $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set -d $REPO/gpurun_out/pmc$i -o run --output-format csv -- python3 $REPO/bench.py --steps 2 --warmup 1 --rpc 0 ${BENCH_ARGS:-} > $REPO/gpurun_out/pmc$i.log 2>&1 || { echo "set $i failed rc=$?"; tail -5 $REPO/gpurun_out/pmc$i.log; exit 1; }
done
echo done
