#!/bin/bash
# A/B of post-processing builds (tools/bin/post_bench_<v>, csrc/tools/post_bench.hip):
# wall time per call on flat / planted / noisy maps and on the bench model's own label
# maps (dumped by scripts/label_stats.py), then per-kernel averages on the bench maps
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
O=gpurun_out/post_ab
mkdir -p $O
timeout -k 10 200 python scripts/label_stats.py $REPO/$O/bench_labels.bin > $O/label_stats.txt 2>&1 || { tail -5 $O/label_stats.txt; exit 3; }
cat $O/label_stats.txt
for v in ${VERS:-old new}; do
  echo "== $v"
  timeout -k 10 60 tools/bin/post_bench_$v 50 $O/bench_labels.bin || exit 1
done
for d in ${DBGS:-}; do echo "== s5 SSA_POST_DBG=$d"; SSA_POST_DBG=$d timeout -k 10 60 tools/bin/post_bench_s5 50 $O/bench_labels.bin || exit 1; done
for q in ${QBS:-}; do echo "== new SSA_QUAD_BLOCKS=$q"; SSA_QUAD_BLOCKS=$q timeout -k 10 60 tools/bin/post_bench_new 50 $O/bench_labels.bin || exit 1; done
cd /tmp && export TMPDIR=/tmp
for v in ${VERS:-old new}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $REPO/$O/$v -o run --output-format csv -- $REPO/tools/bin/post_bench_$v 20 $REPO/$O/bench_labels.bin only > $REPO/$O/$v.log 2>&1 || exit 2
  echo "== $v kernels (bench label maps)"
  python3 - "$(ls $REPO/$O/$v/*/run_kernel_stats.csv 2>/dev/null || ls $REPO/$O/$v/run_kernel_stats.csv)" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:40]:40s} calls {int(r['Calls']):5d} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
