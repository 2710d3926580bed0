#!/bin/bash
# Grid-cap sweep of the device post-processing (debug post_bench build, SSA_CCL_GRID /
# SSA_ACC_GRID env): bash scripts/post_grid.sh OUTDIR "c:a c:a ..." (0 = one block per tile)
set -o pipefail
cd "$(dirname "$0")/.."
O=$1; shift
mkdir -p $O
[ -f /tmp/ssa_maps.bin ] || timeout -k 10 300 python scripts/label_stats.py /tmp/ssa_maps.bin > $O/label_stats.txt 2>&1 \
  || { tail -5 $O/label_stats.txt; exit 7; }
for spec in $1; do
  c=${spec%%:*}; a=${spec#*:}
  env SSA_CCL_GRID=$c SSA_ACC_GRID=$a SSA_POST_STAGEWISE=1 timeout -k 10 180 tools/bin/pb_base ${POST_REPS:-30} /tmp/ssa_maps.bin 1 \
    > $O/grid_${c}_${a}.txt 2>&1 || { tail -5 $O/grid_${c}_${a}.txt; exit 7; }
  echo "== ccl_grid=$c acc_grid=$a"; cat $O/grid_${c}_${a}.txt
done
