#!/bin/bash
# Config 2 (batch 1): bench + kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 300 python bench.py --batch 1 --steps 400 --warmup 40 --rpc 0 > gpurun_out/b1_bench.json 2> gpurun_out/b1_bench.err || { tail -20 gpurun_out/b1_bench.err; exit 3; }
cat gpurun_out/b1_bench.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/b1_prof -o run --output-format csv -- python3 $REPO/bench.py --batch 1 --steps 20 --warmup 5 --rpc 0 > $REPO/gpurun_out/b1_prof.log 2>&1
echo "prof rc=$?"
