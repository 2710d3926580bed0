#!/bin/bash
# poison runs: which kernel reads on-chip / global state it did not write
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/debug_poison.py 2 257 160x120 ABCD > gpurun_out/poison_b2.txt 2>&1 || exit $?
timeout -k 10 400 python -u scripts/debug_poison.py 8 513 640x480 ABCD > gpurun_out/poison_b8.txt 2>&1
