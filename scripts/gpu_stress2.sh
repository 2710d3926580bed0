#!/bin/bash
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out
ONLY=32 DETAIL=1 timeout -k 10 300 python -u scripts/debug_stress.py 2 257 160x120 400 2 leaf > gpurun_out/stress_pool.txt 2>&1
