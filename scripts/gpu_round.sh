#!/bin/bash
# conv microbench (CONV_ARGS) + full GPU tests + bench + kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 300 python scripts/bench_conv.py ${CONV_ARGS:---only mnv2 --variants 1,4,7} > gpurun_out/r_conv.txt 2>&1 || { tail -5 gpurun_out/r_conv.txt; exit 1; }
cat gpurun_out/r_conv.txt | grep -v amdgpu.ids
bash scripts/gpu_quick.sh
