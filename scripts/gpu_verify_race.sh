#!/bin/bash
# round 3: concurrency correctness with packed-f32 off, at the test shape and the headline
set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out
RACE_B=32 RACE_S=513 RACE_CAM=640x480 timeout -k 10 400 python -u scripts/debug_race.py 100 "" > gpurun_out/race_b32.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 300 -k "model_parts or records_match or bound_input" -rxX > gpurun_out/race_tests.txt 2>&1
