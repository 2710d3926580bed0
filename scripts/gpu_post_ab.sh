#!/bin/bash
# A/B of post-processing builds (tools/bin/post_bench_<v>, csrc/tools/post_bench.hip):
# wall time per call on flat / planted / noisy maps, then per-kernel averages
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
O=gpurun_out/post_ab
mkdir -p $O
for v in ${VERS:-old new}; do
  echo "== $v"
  timeout -k 10 60 tools/bin/post_bench_$v 50 || exit 1
done
for d in ${DBGS:-}; do echo "== new SSA_POST_DBG=$d"; SSA_POST_DBG=$d timeout -k 10 60 tools/bin/post_bench_new 50 || exit 1; done
cd /tmp && export TMPDIR=/tmp
for v in ${VERS:-old new}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $REPO/$O/$v -o run --output-format csv -- $REPO/tools/bin/post_bench_$v 20 > $REPO/$O/$v.log 2>&1 || exit 2
  echo "== $v kernels (avg us over the 3 map kinds)"
  python3 - "$(ls $REPO/$O/$v/*/run_kernel_stats.csv 2>/dev/null || ls $REPO/$O/$v/run_kernel_stats.csv)" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:40]:40s} calls {int(r['Calls']):5d} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
