#!/bin/bash
# round 3 evidence: long race runs, RCCL world-1 path, B=1 trace, config 4 (>=50 steps)
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python -u scripts/debug_race.py 1000 "" > $O/race_b2.txt 2>&1 || exit $?
RACE_B=32 RACE_S=513 RACE_CAM=640x480 timeout -k 10 400 python -u scripts/debug_race.py 334 "" > $O/race_b32.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 300 -k "rccl_world1 or records_match or concurrent or function_of or rejects" > $O/tests.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --arch resnet50 --input_size 1025 --camera 2048x1024 --dtype int8 --batch 8 --steps 60 --warmup 10 --rpc 0 > $O/c4_int8.json 2> $O/c4_int8.err || exit $?
timeout -k 10 300 python bench.py --arch resnet50 --input_size 1025 --camera 2048x1024 --batch 8 --steps 60 --warmup 10 --rpc 0 > $O/c4_bf16.json 2> $O/c4_bf16.err || exit $?
cd /tmp && export TMPDIR=/tmp
SSA_SLOT_PARALLEL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$O/b1_prof -o run --output-format csv -- python3 $REPO/bench.py --batch 1 --steps 20 --warmup 5 --lag 1 --rpc 0 > $REPO/$O/b1_prof.log 2>&1 || exit $?
SSA_SLOT_PARALLEL=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/$O/c4_prof -o run --output-format csv -- python3 $REPO/bench.py --arch resnet50 --input_size 1025 --camera 2048x1024 --dtype int8 --batch 8 --steps 4 --warmup 2 --lag 1 --rpc 0 > $REPO/$O/c4_prof.log 2>&1
