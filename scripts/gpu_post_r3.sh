#!/bin/bash
# round 3 post-processing rework (k_accum = quads + tree + hist, root list instead of
# k_select, no k_compress, counters zeroed in k_ccl_local, fallback merge inside
# k_ccl_merge): full GPU suite, driver-window and 100-step bench, sequential kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
O=gpurun_out/post_r3
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt

for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20_$i.json 2> $O/bench_20_$i.err || exit 2; cut -c1-200 $O/bench_20_$i.json; done
timeout -k 10 300 python bench.py --steps 100 --warmup 20 > $O/bench_100.json 2> $O/bench_100.err || exit 3
cut -c1-200 $O/bench_100.json
cd /tmp && export TMPDIR=/tmp
SSA_SLOT_PARALLEL=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/$O/seq -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --lag 1 --rpc 0 > $REPO/$O/seq.log 2>&1 || exit 5
cd $REPO
python3 scripts/layer_times.py $(ls $O/seq/*/run_kernel_trace.csv 2>/dev/null || ls $O/seq/run_kernel_trace.csv) > $O/layer_times.txt
tail -20 $O/layer_times.txt
