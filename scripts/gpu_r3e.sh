#!/bin/bash
# round 3 final consolidation (post rework + ASPP v18 at B=1): full GPU suite, driver-window bench (20/5) x2, 100-step bench,
# batch 1, then a kernel trace of the headline step (sequential model for per-kernel times)
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
# concurrent plan copies (slot-parallel default) with the round-3 kernels: label maps must
# equal the sequential reference
timeout -k 10 300 python -u scripts/debug_race.py 500 "" > $O/race_b2.txt 2>&1 || { tail -5 $O/race_b2.txt; exit 6; }
RACE_B=32 RACE_S=513 RACE_CAM=640x480 timeout -k 10 400 python -u scripts/debug_race.py 150 "" > $O/race_b32.txt 2>&1 || { tail -5 $O/race_b32.txt; exit 7; }
grep -h "mismatch" $O/race_b2.txt $O/race_b32.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default_$i.json 2> $O/bench_default_$i.err || exit 2
  cut -c1-160 $O/bench_default_$i.json
done
timeout -k 10 300 python bench.py --steps 100 --warmup 20 > $O/bench_100.json 2> $O/bench_100.err || exit 3
timeout -k 10 300 python bench.py --batch 1 --steps 400 --warmup 50 --rpc 0 > $O/bench_b1.json 2> $O/bench_b1.err || exit 4
cut -c1-160 $O/bench_100.json $O/bench_b1.json
cd /tmp && export TMPDIR=/tmp
SSA_SLOT_PARALLEL=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/$O/seq -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --lag 1 --rpc 0 > $REPO/$O/seq.log 2>&1 || exit 5
cd $REPO
python3 scripts/layer_times.py $(ls $O/seq/*/run_kernel_trace.csv 2>/dev/null || ls $O/seq/run_kernel_trace.csv) > $O/layer_times.txt
tail -45 $O/layer_times.txt
