#!/bin/bash
# Kernel-trace profiles of selected bench configs: gpurun_out/pc_<tag>/
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
prof() { local tag=$1; shift; echo "== $tag"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/pc_$tag -o run --output-format csv -- python3 $REPO/bench.py --rpc 0 "$@" > $REPO/gpurun_out/pc_$tag.log 2>&1; local rc=$?; tail -c 600 $REPO/gpurun_out/pc_$tag.log; return $rc; }
prof r50_int8 --arch resnet50 --dtype int8 --input_size 1025 --camera 2048x1024 --batch 8 --steps 3 --warmup 2 && \
prof r50_bf16 --arch resnet50 --dtype bf16 --input_size 1025 --camera 2048x1024 --batch 8 --steps 3 --warmup 2 && \
prof b1_graph --batch 1 --steps 20 --warmup 5 && \
prof b1_nograph --batch 1 --steps 20 --warmup 5 --no-graph
