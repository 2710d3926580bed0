#!/bin/bash
# Round-2 GPU iteration: selected GPU tests (TESTS=-k expr), headline bench with the
# autotune log, and (PROF=1) a rocprofv3 kernel trace of a short bench.
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1 SSA_LOG_AUTOTUNE=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x -k "$TESTS" --timeout 300 --timeout-method thread > gpurun_out/r2_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/r2_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --steps ${STEPS:-40} --warmup 5 --rpc ${RPC:-500} ${BENCH_ARGS:-} > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err || { grep -v "^frame" gpurun_out/r2_bench.err | tail -20; exit 3; }
  cat gpurun_out/r2_bench.json; grep autotune gpurun_out/r2_bench.err | head -40
fi
if [ "${PROF:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/r2_prof -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --rpc 0 ${BENCH_ARGS:-} > $REPO/gpurun_out/r2_prof.log 2>&1
  echo "prof rc=$?"
fi
exit 0
