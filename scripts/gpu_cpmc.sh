#!/bin/bash
# PMC on single conv shapes (SHAPES env, space separated), variant V (default 1)
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
for sh in ${SHAPES:-b15_exp}; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_LDS" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
             "FETCH_SIZE WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $set -d $REPO/gpurun_out/cpmc_${sh}_$i -o run --output-format csv -- python3 $REPO/scripts/bench_conv.py --shape $sh --variants ${V:-1} --reps 2 > $REPO/gpurun_out/cpmc_${sh}_$i.log 2>&1 || { echo "pmc $sh $i failed"; tail -3 $REPO/gpurun_out/cpmc_${sh}_$i.log; exit 2; }
  done
done
echo done
