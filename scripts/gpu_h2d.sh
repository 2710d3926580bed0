#!/bin/bash
# SSA_H2D_ON_SLOT A/B: frames uploaded on the slot's model stream vs a copy stream
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
SSA_H2D_ON_SLOT=1 timeout -k 10 300 python -u -m pytest tests/ -q -m gpu -x -k "dp_pipeline_records or slot or engine_bound" --timeout 120 --timeout-method thread > gpurun_out/h2d_tests.log 2>&1 || { tail -30 gpurun_out/h2d_tests.log; exit 1; }
tail -2 gpurun_out/h2d_tests.log
: > gpurun_out/h2d_ab.txt
for i in 1 2; do
  for cfg in "0 32" "1 32" "0 1" "1 1"; do
    set -- $cfg
    steps=100; [ $2 = 1 ] && steps=400
    SSA_H2D_ON_SLOT=$1 timeout -k 10 300 python bench.py --batch $2 --steps $steps --warmup 20 --rpc 0 > gpurun_out/h2d.json 2> gpurun_out/h2d.err || { tail -20 gpurun_out/h2d.err; exit 3; }
    python -c "import json; d=json.load(open('gpurun_out/h2d.json')); print('h2d_on_slot=$1 batch=$2', d['value'], d['ms_per_step'])" | tee -a gpurun_out/h2d_ab.txt
  done
done
