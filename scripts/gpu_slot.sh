#!/bin/bash
# slot-parallel vs 2 model parts: pipeline record tests + A/B benches (B=32, B=1)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu -x -k "dp_pipeline or engine_bound" --timeout 120 --timeout-method thread > gpurun_out/sl_tests.log 2>&1 || { tail -30 gpurun_out/sl_tests.log; exit 1; }
tail -2 gpurun_out/sl_tests.log
: > gpurun_out/slot_ab.txt
for i in 1 2; do
  for mode in parts2 slot b1 b1slot; do
    case $mode in
      parts2) env="SSA_MODEL_PARTS=2"; args="";;
      slot) env="SSA_SLOT_PARALLEL=1 SSA_MODEL_PARTS=1"; args="";;
      b1) env=""; args="--batch 1 --steps 400 --warmup 40";;
      b1slot) env="SSA_SLOT_PARALLEL=1"; args="--batch 1 --steps 400 --warmup 40";;
    esac
    env $env timeout -k 10 300 python bench.py --steps 100 --warmup 10 --rpc 0 $args > gpurun_out/sl.json 2> gpurun_out/sl.err || { tail -20 gpurun_out/sl.err; exit 3; }
    python -c "import json; d=json.load(open('gpurun_out/sl.json')); print('$mode', d['value'], d['ms_per_step'])" | tee -a gpurun_out/slot_ab.txt
  done
done
