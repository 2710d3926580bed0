#!/bin/bash
# pipeline depth A/B (SSA_PIPE_LAG 1 vs 2: two vs three staging slots / steps in flight)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
SSA_PIPE_LAG=2 timeout -k 10 300 python -u -m pytest tests/ -q -m gpu -x -k "dp_pipeline_records or slot" --timeout 120 --timeout-method thread > gpurun_out/lag_tests.log 2>&1 || { tail -30 gpurun_out/lag_tests.log; exit 1; }
tail -2 gpurun_out/lag_tests.log
: > gpurun_out/lag_ab.txt
for i in 1 2; do
  for cfg in "1 32" "2 32" "1 1" "2 1"; do
    set -- $cfg
    steps=100; [ $2 = 1 ] && steps=400
    SSA_PIPE_LAG=$1 timeout -k 10 300 python bench.py --batch $2 --steps $steps --warmup 20 --rpc 0 > gpurun_out/lag.json 2> gpurun_out/lag.err || { tail -20 gpurun_out/lag.err; exit 3; }
    python -c "import json; d=json.load(open('gpurun_out/lag.json')); print('lag=$1 batch=$2', d['value'], d['ms_per_step'])" | tee -a gpurun_out/lag_ab.txt
  done
done
