#!/bin/bash
# fused_ir_stream: numerics tests + microbenchmark (+ timeline) per 33x33 block shape
set -o pipefail
export SSA_NO_AUTOBUILD=1
O=gpurun_out/stream
mkdir -p $O
rm -f $O/trace.txt
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k "fused_ir_stream" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for b in ${TRACE_BLOCKS:-7 11 14 16}; do
  timeout -k 10 120 python scripts/bench_span.py --stream --only $b --S 8 --trace --reps 30 >> $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 2; }
done
grep -v amdgpu $O/trace.txt
