#!/bin/bash
# Round-end style verification: upsample microbench, GPU tests, smoke(), headline bench.
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1 SSA_LOG_AUTOTUNE=1
timeout -k 10 120 env PYTHONPATH=$REPO python scripts/bench_upsample.py > gpurun_out/v_ups.txt 2>&1 || { cat gpurun_out/v_ups.txt; exit 3; }
cat gpurun_out/v_ups.txt
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/v_tests.log 2>&1
rc=$?
tail -3 gpurun_out/v_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1 || { tail gpurun_out/v_smoke.log; exit 6; }
tail -1 gpurun_out/v_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/v_bench.json 2> gpurun_out/v_bench.err || { tail gpurun_out/v_bench.err; exit 4; }
cat gpurun_out/v_bench.json; grep "autotune.*upsample" gpurun_out/v_bench.err
