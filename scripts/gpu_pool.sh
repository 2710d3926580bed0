#!/bin/bash
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/debug_pool.py 1600 2 > gpurun_out/pool_nopk_m2.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/debug_race.py 300 "" > gpurun_out/race_nopk.txt 2>&1 || exit $?
timeout -k 10 400 python -u scripts/debug_stress.py 2 257 160x120 300 2 leaf > gpurun_out/stress_nopk.txt 2>&1
