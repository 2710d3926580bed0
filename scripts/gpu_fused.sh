#!/bin/bash
# fused-IR microbench + PMC on one block, post-processing tests, bench
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_hip_kernels.py -q -x -k "post or ccl or fused or stream_group or engine" > gpurun_out/f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/f_tests.log; [ $rc -ne 0 ] && { grep -n "Error\|assert" gpurun_out/f_tests.log | head; exit $rc; }
for b in 1 2 11 14 16; do timeout -k 10 120 python scripts/bench_fused.py --block $b --tiles 5x11,11x11,8x16,4x16 || exit 1; done 2>&1 | tee gpurun_out/f_bench.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $REPO/gpurun_out/fpmc1 -o run --output-format csv -- python3 $REPO/scripts/bench_fused.py --block 14 --tiles 5x11 --reps 3 > $REPO/gpurun_out/fpmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $REPO/gpurun_out/fpmc2 -o run --output-format csv -- python3 $REPO/scripts/bench_fused.py --block 14 --tiles 5x11 --reps 3 > $REPO/gpurun_out/fpmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM -d $REPO/gpurun_out/fpmc3 -o run --output-format csv -- python3 $REPO/scripts/bench_fused.py --block 14 --tiles 5x11 --reps 3 > $REPO/gpurun_out/fpmc3.log 2>&1 || exit 4
cd $REPO
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rpc 500 > gpurun_out/f_bench.json 2> gpurun_out/f_bench.err || exit 5
cat gpurun_out/f_bench.json
