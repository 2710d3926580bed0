#!/bin/bash
# The round-3 packed-f32 finding, re-checked on the current tree: the
# aspp_pool leaf under plan-copy noise (scripts/debug_pool.py, mode 2) and the concurrent
# plan determinism check (scripts/debug_race.py), each with the shipped build (packed-f32
# VALU compiled out) and with a packed-f32 build of the same sources
# (SSA_PACKED_F32=1 SSA_HIP_OUT=tools/bin/_hip_pk.so python -m semantic_segmentation_server_amd.ops.build).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:?outdir}; N=${2:-800}
mkdir -p $O
export SSA_NO_AUTOBUILD=1
for b in nopk pk; do
  so=""; [ $b = pk ] && so=tools/bin/_hip_pk.so
  SSA_HIP_SO=$so timeout -k 10 300 python -u scripts/debug_pool.py $N 2 > $O/pool_$b.txt 2>&1 || { tail -5 $O/pool_$b.txt; exit 1; }
  echo "pool $b: $(grep '^mode' $O/pool_$b.txt)"
  SSA_HIP_SO=$so timeout -k 10 400 python -u scripts/debug_race.py > $O/race_$b.txt 2>&1 || { tail -5 $O/race_$b.txt; exit 1; }
  echo "race $b: $(tail -1 $O/race_$b.txt)"
done
