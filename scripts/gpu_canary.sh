#!/bin/bash
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/debug_lds_canary.py 2 257 160x120 50 > gpurun_out/canary_b2.txt 2>&1 || exit $?
ALL_VARIANTS=1 timeout -k 10 300 python -u scripts/debug_lds_canary.py 2 257 160x120 30 > gpurun_out/canary_b2_all.txt 2>&1
