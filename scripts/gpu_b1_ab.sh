#!/bin/bash
# Batch-1 bench A/B of two autotune pick files, interleaved on one box:
#   TUNE_A=assets/tune_mi355x.json TUNE_B=<candidate picks> bash scripts/gpu_b1_ab.sh
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out/b1ab
for i in 1 2; do
for t in ${TUNE_A:-assets/tune_mi355x.json} ${TUNE_B:?candidate pick file}; do
  SSA_TUNE_FILE=$PWD/$t timeout -k 10 200 python bench.py --batch 1 --steps 400 --warmup 50 --rpc 0 > gpurun_out/b1ab/b1_$i.json 2> gpurun_out/b1ab/b1_$i.err || exit 1
  echo "$t $(python -c "import json;d=json.load(open('gpurun_out/b1ab/b1_$i.json'));print(d['ms_per_step'])")"
done; done
