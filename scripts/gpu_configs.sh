#!/bin/bash
# Benchmark every BASELINE.json config that fits one GPU; JSON lines -> gpurun_out/configs.jsonl
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
OUT=gpurun_out/configs.jsonl
: > $OUT
run() { local tag=$1; shift; echo "== $tag" >&2; timeout -k 10 400 python bench.py "$@" 2> gpurun_out/cfg_$tag.err | sed "s/^{/{\"tag\": \"$tag\", /" >> $OUT; local rc=$?; [ $rc -ne 0 ] && { grep -v "^frame" gpurun_out/cfg_$tag.err | tail -5; }; return $rc; }
run c3_mnv2_b32 --steps 30 --warmup 5 --rpc 2000 && \
run c2_mnv2_b1 --batch 1 --steps 200 --warmup 20 --rpc 0 && \
run c2_mnv2_b1_nograph --batch 1 --steps 100 --warmup 10 --rpc 0 --no-graph && \
run c5_mnv2_4streams --batch 32 --streams 4 --steps 30 --warmup 5 --rpc 0 && \
run c3_mnv2_b64 --batch 64 --steps 20 --warmup 5 --rpc 0 && \
run c4_r50_int8_1025 --arch resnet50 --dtype int8 --input_size 1025 --camera 2048x1024 --batch 8 --steps 10 --warmup 3 --rpc 0 && \
run c4_r50_bf16_1025 --arch resnet50 --dtype bf16 --input_size 1025 --camera 2048x1024 --batch 8 --steps 10 --warmup 3 --rpc 0
rc=$?
cat $OUT | cut -c1-420
exit $rc
