#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 per counter set; no trace modes).
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "== pmc set $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set -d $REPO/gpurun_out/pmc$i -o run --output-format csv -- python3 $REPO/bench.py --steps 2 --warmup 1 --rpc 0 ${BENCH_ARGS:-} > $REPO/gpurun_out/pmc$i.log 2>&1 || { echo "set $i failed rc=$?"; tail -5 $REPO/gpurun_out/pmc$i.log; exit 1; }
done
echo done
