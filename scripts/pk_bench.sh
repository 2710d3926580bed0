#!/bin/bash
# Headline bench, shipped build (packed-f32 VALU compiled out) vs a packed-f32 build of the
# same sources (tools/bin/_hip_pk.so, loaded through SSA_HIP_SO), interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:?outdir}; R=${2:-2}
mkdir -p $O
export SSA_NO_AUTOBUILD=1
for r in $(seq 1 $R); do
  for b in nopk pk; do
    so=""; [ $b = pk ] && so=tools/bin/_hip_pk.so
    SSA_HIP_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 5 $BENCH_ARGS > $O/pkb_$b$r.json 2> $O/pkb_$b$r.err \
      || { echo "$b failed"; tail -5 $O/pkb_$b$r.err; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/pkb_$b$r.json') if l.startswith('{')][-1]); print('$b$r', d['value'], d['ms_per_step'])"
  done
done
