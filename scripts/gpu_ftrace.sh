#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out
for b in 2 11 14; do timeout -k 10 120 python scripts/bench_fused.py --block $b --tiles 11x11 --trace || exit 1; done 2>&1 | tee gpurun_out/ftrace.txt
