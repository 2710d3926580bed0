#!/bin/bash
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/debug_pool.py 600 0 > gpurun_out/pool_m0.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/debug_pool.py 600 2 > gpurun_out/pool_m2.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/debug_pool.py 600 1 > gpurun_out/pool_m1.txt 2>&1
