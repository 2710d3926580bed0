#!/bin/bash
# World-size-1 A/B of the RCCL data path: the default (no group, local
# ingest, host record gather) against a real RCCL group (SSA_FORCE_PG=1) with the record
# gather and / or the frame scatter on the pipeline's own streams (parallel/rccl.py), and
# the same through torch.distributed's internal stream (SSA_RCCL_TORCH=1). Interleaved
# rounds in one call: bash scripts/rccl_ab.sh OUTDIR [ROUNDS]
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:?outdir}; R=${2:-2}
mkdir -p $O
export SSA_NO_AUTOBUILD=1 MASTER_ADDR=127.0.0.1
run() {  # run <tag> <env...> -- <bench args>
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rpc 0 $BA > $O/$tag.json 2> $O/$tag.err \
    || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python -c "import json,sys; d=json.loads([l for l in open('$O/$tag.json') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'], d.get('host_ms_per_step'))"
}
for r in $(seq 1 $R); do
  echo "round $r"
  BA="" run default$r SSA_X=0 || exit 1
  BA="--gather rccl" run gather_stream$r SSA_FORCE_PG=1 MASTER_PORT=2960$r || exit 1
  BA="--gather rccl" run gather_torch$r SSA_FORCE_PG=1 SSA_RCCL_TORCH=1 MASTER_PORT=2961$r || exit 1
  BA="--ingest scatter" run scatter_stream$r SSA_FORCE_PG=1 MASTER_PORT=2962$r || exit 1
  BA="--ingest scatter" run scatter_torch$r SSA_FORCE_PG=1 SSA_RCCL_TORCH=1 MASTER_PORT=2963$r || exit 1
  BA="--ingest scatter --gather rccl" run scatter_gather_stream$r SSA_FORCE_PG=1 MASTER_PORT=2964$r || exit 1
done
