#!/bin/bash
# round 3 (re-entry): GPU suite + default headline bench on the rebuilt tree
set -o pipefail
export SSA_NO_AUTOBUILD=1
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default_$i.json 2> $O/bench_default_$i.err || exit $?
done
timeout -k 10 300 python bench.py --batch 1 --steps 400 --warmup 50 --rpc 0 > $O/bench_b1.json 2> $O/bench_b1.err || exit $?
for b in 7 11 14 16; do
  timeout -k 10 120 python scripts/bench_span.py --only $b --S 8 --trace --reps 20 >> $O/span_trace.txt 2>&1 || exit $?
done
