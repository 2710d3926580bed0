#!/bin/bash
set -o pipefail
export SSA_NO_AUTOBUILD=1
O=gpurun_out/stream
mkdir -p $O
for b in 7 11 13 14; do
  timeout -k 10 120 python scripts/bench_span.py --stream --only $b --S 8 --trace --reps 20 >> $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 2; }
done
grep -v amdgpu $O/trace.txt
