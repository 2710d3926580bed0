#!/bin/bash
# Round-2 config runs: multistream test, config 5 (4 streams x 8 frames, one batched step),
# config 2 (batch 1) bench + kernel trace, and the served loop (bench.py --serve).
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -q -x -k "multistream_batched or stream_group" --timeout 200 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { tail -30 gpurun_out/c_tests.log; exit 1; }
tail -1 gpurun_out/c_tests.log
timeout -k 10 300 python bench.py --streams 4 --steps 60 --warmup 10 --rpc 300 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
tail -1 gpurun_out/c5.json
timeout -k 10 300 python bench.py --batch 1 --steps 300 --warmup 20 --rpc 0 > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -5 gpurun_out/c2.err; exit 1; }
tail -1 gpurun_out/c2.json
timeout -k 10 300 python bench.py --serve --steps 100 --warmup 10 --rpc 500 > gpurun_out/serve.json 2> gpurun_out/serve.err || { tail -5 gpurun_out/serve.err; exit 1; }
tail -1 gpurun_out/serve.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/c2_prof -o run --output-format csv -- python3 $REPO/bench.py --batch 1 --steps 20 --warmup 5 --rpc 0 > $REPO/gpurun_out/c2_prof.log 2>&1
echo "prof rc=$?"
