#!/bin/bash
# GPU validation: kernel goldens + model + graph tests, a short HIP bench, and a
# rocprofv3 kernel-stats profile of the bench.
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
timeout -k 10 600 python -m pytest tests/ -q -m gpu -s > gpurun_out/hip_tests.log 2>&1
rc=$?
tail -15 gpurun_out/hip_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rpc 1000 > gpurun_out/hip_bench.json 2> gpurun_out/hip_bench.err || { grep -v "^frame" gpurun_out/hip_bench.err | tail; exit 3; }
cat gpurun_out/hip_bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rpc 0 --batch 1 > gpurun_out/hip_bench_b1.json 2>/dev/null && cat gpurun_out/hip_bench_b1.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/prof_hip -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --rpc 0 > $REPO/gpurun_out/prof_hip.log 2>&1
echo "prof rc=$?"
exit $rc
