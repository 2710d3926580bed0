#!/bin/bash
# World-size-8 rehearsal of the driver's scaling bench on ONE GPU: 8 ranks share the card
# (SSA_SHARE_GPU=1, gloo group). Throughput is meaningless (one GPU); this checks that the
# 8-rank bench path (gather to rank 0, hub, RPC under load, JSON line) completes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1 SSA_SHARE_GPU=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 8 --steps 10 --warmup 3 --rpc 300 > gpurun_out/s8.json 2> gpurun_out/s8.err || { grep -v "^\[Gloo\]" gpurun_out/s8.err | tail -30; exit 5; }
cat gpurun_out/s8.json
