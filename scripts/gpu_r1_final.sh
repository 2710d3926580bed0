#!/bin/bash
# Upsample variant microbench + kernel tests + bench + profile + 2-rank shared-GPU bench rehearsal.
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1 SSA_LOG_AUTOTUNE=1
timeout -k 10 120 env PYTHONPATH=$REPO python scripts/bench_upsample.py > gpurun_out/f_ups.txt 2>&1 || { cat gpurun_out/f_ups.txt; exit 3; }
cat gpurun_out/f_ups.txt
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x -s --timeout 120 --timeout-method thread > gpurun_out/f_tests.log 2>&1
rc=$?
tail -4 gpurun_out/f_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --rpc 500 > gpurun_out/f_bench.json 2> gpurun_out/f_bench.err || { tail gpurun_out/f_bench.err; exit 4; }
cat gpurun_out/f_bench.json; grep "autotune.*upsample" gpurun_out/f_bench.err
SSA_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29577 bench.py --gpus 2 --steps 10 --warmup 3 --rpc 300 > gpurun_out/f_dp2.json 2> gpurun_out/f_dp2.err || { tail -20 gpurun_out/f_dp2.err; exit 5; }
cat gpurun_out/f_dp2.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $REPO/gpurun_out/f_prof -o run --output-format csv -- python3 $REPO/bench.py --steps 5 --warmup 2 --rpc 0 > $REPO/gpurun_out/f_prof.log 2>&1
echo "prof rc=$?"
