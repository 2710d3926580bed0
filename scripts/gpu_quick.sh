#!/bin/bash
# Quick GPU check: GPU tests + bench (+ optional profile with PROF=1).
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1 SSA_LOG_AUTOTUNE=1
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x -s > gpurun_out/q_tests.log 2>&1
rc=$?
tail -6 gpurun_out/q_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rpc 500 > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || { grep -v "^frame" gpurun_out/q_bench.err | tail; exit 3; }
cat gpurun_out/q_bench.json; grep autotune gpurun_out/q_bench.err | head -20
if [ "${PROF:-1}" = "1" ]; then
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/q_prof -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --rpc 0 > $REPO/gpurun_out/q_prof.log 2>&1
echo "prof rc=$?"
fi
exit $rc
