#!/bin/bash
# round 3: GPU tests + headline A/B (slot-parallel default vs off), packed-f32 off
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out/r3a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3a/pytest.txt 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rpc 300 > gpurun_out/r3a/bench_default_$i.json 2> gpurun_out/r3a/bench_default_$i.err || exit $?
done
SSA_SLOT_PARALLEL=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rpc 0 > gpurun_out/r3a/bench_noslot.json 2> gpurun_out/r3a/bench_noslot.err || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --lag 2 --rpc 0 > gpurun_out/r3a/bench_lag2.json 2> gpurun_out/r3a/bench_lag2.err || exit $?
timeout -k 10 300 python bench.py --batch 1 --steps 400 --warmup 50 --rpc 0 > gpurun_out/r3a/bench_b1.json 2> gpurun_out/r3a/bench_b1.err || exit $?
timeout -k 10 300 python bench.py --batch 1 --steps 400 --warmup 50 --lag 2 --rpc 0 > gpurun_out/r3a/bench_b1_lag2.json 2> gpurun_out/r3a/bench_b1_lag2.err
