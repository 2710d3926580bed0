#!/bin/bash
# Re-time selected plan steps (ONLY=comma list) on top of the committed picks for the batch
# sizes in BATCHES (default "32 1"), optional GPU tests (TESTS=-k expr), then bench.
set -o pipefail
export SSA_NO_AUTOBUILD=1
O=gpurun_out/retune
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "$TESTS" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
  tail -1 $O/tests.txt
fi
cp assets/tune_mi355x.json $O/tune.json
for B in ${BATCHES:-32 1}; do
  SSA_TUNE_FILE=$PWD/$O/tune.json SSA_RETUNE_ONLY=$ONLY SSA_LOG_AUTOTUNE=1 timeout -k 10 300 python bench.py --batch $B --steps 20 --warmup 5 --rpc 0 > $O/tune_$B.json 2> $O/tune_$B.err || { tail -5 $O/tune_$B.err; exit 2; }
  grep "autotune B=" $O/tune_$B.err | grep -v "picks from" | cut -c1-500
done
for B in ${BATCHES:-32 1}; do
  SSA_TUNE_FILE=$PWD/$O/tune.json timeout -k 10 300 python bench.py --batch $B --steps $([ $B = 1 ] && echo 400 || echo 100) --warmup 20 > $O/bench_$B.json 2> $O/bench_$B.err || { tail -5 $O/bench_$B.err; exit 3; }
  cut -c1-200 $O/bench_$B.json
done
