#!/bin/bash
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out/tl
timeout -k 10 200 python -u scripts/lag_timeline.py 2 5 20 > gpurun_out/tl/lag2_k.txt 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lag 2 --rpc 0 > gpurun_out/tl/bench_lag2_$i.json 2> gpurun_out/tl/bench_lag2_$i.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lag 1 --rpc 0 > gpurun_out/tl/bench_lag1_$i.json 2> gpurun_out/tl/bench_lag1_$i.err || exit $?
done
