#!/bin/bash
# race localisation: baseline reproduction, then per-leaf stress under plan-copy noise
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/debug_race.py 150 "" > gpurun_out/race_base.txt 2>&1 || exit $?
timeout -k 10 400 python -u scripts/debug_stress.py 2 257 160x120 200 2 leaf > gpurun_out/stress_leaf.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/debug_stress.py 2 257 160x120 150 2 seq > gpurun_out/stress_seq.txt 2>&1
