#!/bin/bash
# conv_gemm variant correctness + microbenchmark
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_hip_kernels.py -q -x -k "conv_gemm" > gpurun_out/conv_tests.log 2>&1
rc=$?; tail -5 gpurun_out/conv_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bench_conv.py ${BENCH_ARGS:-} 2>&1 | tee gpurun_out/conv_bench.txt
