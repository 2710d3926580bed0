#!/bin/bash
# batch-1 check: post-processing GPU tests, two batch-1 benches, batch-1 sequential trace
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
O=gpurun_out/b1chk
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "postprocess or records or post" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --batch 1 --steps 400 --warmup 50 --rpc 0 > $O/bench_b1_$i.json 2> $O/bench_b1_$i.err || exit 3
  cut -c1-160 $O/bench_b1_$i.json
done
cd /tmp && export TMPDIR=/tmp
SSA_SLOT_PARALLEL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $REPO/$O/b1seq -o run --output-format csv -- python3 $REPO/bench.py --batch 1 --steps 20 --warmup 5 --lag 1 --rpc 0 > $REPO/$O/b1seq.log 2>&1 || exit 5
cd $REPO
python3 scripts/layer_times.py $(ls $O/b1seq/*/run_kernel_trace.csv 2>/dev/null || ls $O/b1seq/run_kernel_trace.csv) > $O/b1_layer_times.txt
tail -8 $O/b1_layer_times.txt
