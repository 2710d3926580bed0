#!/bin/bash
# round 3: kernel traces of the headline step (sequential model for clean per-kernel
# times; default slot-parallel mode for the stats)
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out/prof_r3
cd /tmp && export TMPDIR=/tmp
SSA_SLOT_PARALLEL=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/prof_r3/seq -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --lag 1 --rpc 0 > $REPO/gpurun_out/prof_r3/seq.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/prof_r3/def -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --rpc 0 > $REPO/gpurun_out/prof_r3/def.log 2>&1
