#!/bin/bash
# Round-2 re-entry: full GPU tests, headline bench (100 steps), kernel trace of a short bench.
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1 SSA_LOG_AUTOTUNE=1
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x ${TEST_ARGS:-} --timeout 120 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/r2c_tests.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  for i in 1 2; do
    timeout -k 10 300 python bench.py --steps 100 --warmup 10 --rpc ${RPC:-300} ${BENCH_ARGS:-} > gpurun_out/r2c_bench$i.json 2> gpurun_out/r2c_bench$i.err || { tail -20 gpurun_out/r2c_bench$i.err; exit 3; }
    cat gpurun_out/r2c_bench$i.json
  done
fi
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/r2c_prof -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --rpc 0 ${BENCH_ARGS:-} > $REPO/gpurun_out/r2c_prof.log 2>&1
  echo "prof rc=$?"
fi
exit 0
