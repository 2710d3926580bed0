#!/bin/bash
# Regenerate the committed plan picks (assets/tune_mi355x.json) on a fresh box: the
# headline B=32 plan and the batch-1 plan, each autotuned 3 times; the picks of the
# fastest of the three runs are kept (timings are noisy, ~2-3 %).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/tune
export SSA_NO_AUTOBUILD=1
for B in 32 1; do
  for k in 1 2 3; do
    rm -f gpurun_out/tune/t_${B}_$k.json
    SSA_TUNE_FILE=$PWD/gpurun_out/tune/t_${B}_$k.json timeout -k 10 300 python bench.py --batch $B --steps $([ $B = 1 ] && echo 300 || echo 60) --warmup 10 --rpc 0 > gpurun_out/tune/b_${B}_$k.json 2> gpurun_out/tune/b_${B}_$k.err || { tail -5 gpurun_out/tune/b_${B}_$k.err; exit 1; }
    tail -1 gpurun_out/tune/b_${B}_$k.json | cut -c1-120
  done
done
