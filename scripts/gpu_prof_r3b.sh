#!/bin/bash
# round 3 (after the stream kernel): kernel traces of the headline step (sequential model
# for clean per-kernel times; default slot-parallel mode for stats + exclusive times)
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
O=gpurun_out/prof_r3b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SSA_SLOT_PARALLEL=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/$O/seq -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --lag 1 --rpc 0 > $REPO/$O/seq.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/$O/def -o run --output-format csv -- python3 $REPO/bench.py --steps 20 --warmup 5 --rpc 0 > $REPO/$O/def.log 2>&1 || exit $?
cd $REPO
python3 scripts/layer_times.py $(ls $O/seq/*/run_kernel_trace.csv 2>/dev/null || ls $O/seq/run_kernel_trace.csv) > $O/layer_times.txt
python3 scripts/exclusive_time.py $(ls $O/def/*/run_kernel_trace.csv 2>/dev/null || ls $O/def/run_kernel_trace.csv) > $O/exclusive.txt
tail -50 $O/layer_times.txt
