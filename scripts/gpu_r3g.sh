#!/bin/bash
# round 3 closing run: full GPU suite, driver-window bench x2, batch-1 bench, batch-1
# sequential kernel trace (per-kernel table of the final tree)
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default_$i.json 2> $O/bench_default_$i.err || exit 2
  cut -c1-160 $O/bench_default_$i.json
done
timeout -k 10 300 python bench.py --batch 1 --steps 400 --warmup 50 --rpc 0 > $O/bench_b1.json 2> $O/bench_b1.err || exit 3
cut -c1-160 $O/bench_b1.json
cd /tmp && export TMPDIR=/tmp
SSA_SLOT_PARALLEL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$O/b1seq -o run --output-format csv -- python3 $REPO/bench.py --batch 1 --steps 20 --warmup 5 --lag 1 --rpc 0 > $REPO/$O/b1seq.log 2>&1 || exit 5
cd $REPO
python3 scripts/layer_times.py $(ls $O/b1seq/*/run_kernel_trace.csv 2>/dev/null || ls $O/b1seq/run_kernel_trace.csv) > $O/b1_layer_times.txt
tail -12 $O/b1_layer_times.txt
