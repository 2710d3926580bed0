#!/bin/bash
# Re-time the grouped ASPP choice (new branch-affine XCD tile orders) on top of the
# committed picks for B=32, then bench with the new picks.
set -o pipefail
export SSA_NO_AUTOBUILD=1
O=gpurun_out/tune_aspp
mkdir -p $O
if [ -f gpurun_out/tune_stream/tune.json ] && [ "${ASPP_FROM_STREAM:-0}" = 1 ]; then cp gpurun_out/tune_stream/tune.json $O/tune.json; else cp assets/tune_mi355x.json $O/tune.json; fi
SSA_TUNE_FILE=$PWD/$O/tune.json SSA_RETUNE_ONLY=aspp.branches SSA_LOG_AUTOTUNE=1 timeout -k 10 300 python bench.py --batch 32 --steps 20 --warmup 5 --rpc 0 > $O/tune_32.json 2> $O/tune_32.err || { tail -5 $O/tune_32.err; exit 1; }
grep "autotune" $O/tune_32.err | grep "aspp.branches" | cut -c1-600
SSA_TUNE_FILE=$PWD/$O/tune.json timeout -k 10 300 python bench.py --batch 32 --steps 100 --warmup 20 > $O/bench_32.json 2> $O/bench_32.err || { tail -5 $O/bench_32.err; exit 2; }
cut -c1-300 $O/bench_32.json
