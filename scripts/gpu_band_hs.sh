#!/bin/bash
# fused_ir_band hs=2 (hidden-split waves): numerics tests + retune of blocks 3-6 + bench
set -o pipefail
export SSA_NO_AUTOBUILD=1
O=gpurun_out/band_hs
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "fused_ir_band" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
cp assets/tune_mi355x.json $O/tune.json
for B in 32 1; do
  SSA_TUNE_FILE=$PWD/$O/tune.json SSA_RETUNE_ONLY=block1,block2,block3,block4,block5,block6 SSA_LOG_AUTOTUNE=1 timeout -k 10 300 python bench.py --batch $B --steps 20 --warmup 5 --rpc 0 > $O/tune_$B.json 2> $O/tune_$B.err || { tail -5 $O/tune_$B.err; exit 2; }
  grep "autotune" $O/tune_$B.err | grep -E "block[1-6]:" | cut -c1-420
done
for B in 32 1; do
  SSA_TUNE_FILE=$PWD/$O/tune.json timeout -k 10 300 python bench.py --batch $B --steps $([ $B = 1 ] && echo 400 || echo 100) --warmup 20 > $O/bench_$B.json 2> $O/bench_$B.err || { tail -5 $O/bench_$B.err; exit 3; }
  cut -c1-200 $O/bench_$B.json
done
