#!/bin/bash
# selected GPU tests (TESTS=-k expr) + span-kernel phase timeline (SPAN_ONLY=block idx list)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x -k "$TESTS" --timeout 120 --timeout-method thread > gpurun_out/st_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/st_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for b in ${SPAN_ONLY:-}; do
  timeout -k 10 120 python scripts/bench_span.py --only $b --S 8 --trace --reps 20 >> gpurun_out/st_span.txt 2>&1 || { tail -5 gpurun_out/st_span.txt; exit 4; }
done
cat gpurun_out/st_span.txt 2>/dev/null | grep -v amdgpu.ids
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --rpc 0 > gpurun_out/st_bench.json 2> gpurun_out/st_bench.err || { tail -20 gpurun_out/st_bench.err; exit 3; }
  cat gpurun_out/st_bench.json
fi
exit 0
