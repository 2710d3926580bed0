#!/bin/bash
# Process-group / record-gather A/B on one GPU + the world-8 gloo gather
# timing on the box's CPUs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_distributed.py -q -s -k gather_cost > gpurun_out/pg_gather8.log 2>&1; grep "gloo gather" gpurun_out/pg_gather8.log
for mode in "default" "force_gloo" "force_rccl_hostgather" "force_rccl_rcclgather"; do
  case $mode in
    default) env="";;
    force_gloo) env="SSA_FORCE_PG=1 SSA_PG_BACKEND=gloo";;
    force_rccl_hostgather) env="SSA_FORCE_PG=1";;
    force_rccl_rcclgather) env="SSA_FORCE_PG=1";;
  esac
  args="--steps 60 --warmup 10 --rpc 0"
  [ $mode = force_rccl_hostgather ] && args="$args --pg nccl"
  [ $mode = force_rccl_rcclgather ] && args="$args --gather rccl"
  env $env timeout -k 10 300 python bench.py $args > gpurun_out/pg_$mode.json 2> gpurun_out/pg_$mode.err || { echo "$mode failed"; tail -5 gpurun_out/pg_$mode.err; exit 1; }
  echo "$mode $(python -c "import json;d=json.load(open('gpurun_out/pg_$mode.json'));print(d['value'], d['config']['process_group'], d['config']['gather'])")"
done
