#!/bin/bash
# SSA_MODEL_PARTS A/B: concurrent sub-batch model graphs (+ per-part post) at B = 32.
# Tunes the part plans into gpurun_out/tune.json (seeded from the committed picks) first.
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu -x -k "dp_pipeline or engine_bound" --timeout 120 --timeout-method thread > gpurun_out/p_tests.log 2>&1 || { tail -30 gpurun_out/p_tests.log; exit 1; }
tail -2 gpurun_out/p_tests.log
cp assets/tune_mi355x.json gpurun_out/tune.json
export SSA_TUNE_FILE=$REPO/gpurun_out/tune.json
for p in 2 4; do
  SSA_MODEL_PARTS=$p SSA_LOG_AUTOTUNE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rpc 0 > gpurun_out/pt$p.json 2> gpurun_out/pt$p.err || { tail -20 gpurun_out/pt$p.err; exit 3; }
done
: > gpurun_out/parts_ab.txt
for i in 1 2; do
  for p in 1 2 4; do
    SSA_MODEL_PARTS=$p timeout -k 10 300 python bench.py --steps 100 --warmup 10 --rpc 0 > gpurun_out/p$p.json 2> gpurun_out/p$p.err || { tail -20 gpurun_out/p$p.err; exit 3; }
    python -c "import json; d=json.load(open('gpurun_out/p$p.json')); print('parts=$p', d['value'], d['ms_per_step'])" | tee -a gpurun_out/parts_ab.txt
  done
done
