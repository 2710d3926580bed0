#!/bin/bash
# Re-time the 33x33 block choices (blocks 7-15, new fused_ir_stream variants) on top of
# the committed picks, for B=32 and B=1; then bench both with the new picks.
set -o pipefail
export SSA_NO_AUTOBUILD=1
O=gpurun_out/tune_stream
mkdir -p $O
cp assets/tune_mi355x.json $O/tune.json
ONLY=${ONLY:-block7,block8,block9,block10,block11,block12,block13,block14,block15,block16}
for B in 32 1; do
  SSA_TUNE_FILE=$PWD/$O/tune.json SSA_RETUNE_ONLY=$ONLY SSA_LOG_AUTOTUNE=1 timeout -k 10 300 python bench.py --batch $B --steps 20 --warmup 5 --rpc 0 > $O/tune_$B.json 2> $O/tune_$B.err || { tail -5 $O/tune_$B.err; exit 1; }
  grep "autotune" $O/tune_$B.err | grep -E "block(7|8|9|1[0-6]):" | sed 's/, dwp[a-z0-9]*\.pw2x3=[0-9.]*us//g' | cut -c1-300
done
for B in 32 1; do
  SSA_TUNE_FILE=$PWD/$O/tune.json timeout -k 10 300 python bench.py --batch $B --steps $([ $B = 1 ] && echo 400 || echo 100) --warmup 20 > $O/bench_$B.json 2> $O/bench_$B.err || { tail -5 $O/bench_$B.err; exit 2; }
  cut -c1-400 $O/bench_$B.json
done
