#!/bin/bash
# Round-2 config sweep: headline, model-only (no contour stats), config 5 (4 streams x 8),
# served loop (--serve), batch 64, batch 1, ResNet-50 int8 / bf16. One JSON line per config in gpurun_out/cfg_r2.jsonl.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export SSA_NO_AUTOBUILD=1
: > gpurun_out/cfg_r2.jsonl
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/cfg_$tag.json 2> gpurun_out/cfg_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/cfg_$tag.err; return 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/cfg_$tag.json')); d['tag']='$tag'; print(json.dumps(d))" >> gpurun_out/cfg_r2.jsonl
  python -c "import json; d=json.load(open('gpurun_out/cfg_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d.get('p50_get_segmented_objects_ms'))"
}
run c3_b32 --steps 100 --warmup 10 --rpc 300 && \
run c3_b32_nopost --steps 100 --warmup 10 --rpc 0 --contour_mode none && \
run c5_s4 --steps 100 --warmup 10 --rpc 0 --streams 4 --batch 32 && \
run c3_serve --steps 100 --warmup 10 --rpc 300 --serve && \
run c3_b64 --steps 50 --warmup 5 --rpc 0 --batch 64 && \
run c2_b1 --steps 400 --warmup 40 --rpc 0 --batch 1 && \
run c4_r50_int8 --arch resnet50 --input_size 1025 --camera 2048x1024 --dtype int8 --batch 8 --steps 10 --warmup 3 --rpc 0 && \
run c4_r50_bf16 --arch resnet50 --input_size 1025 --camera 2048x1024 --batch 8 --steps 10 --warmup 3 --rpc 0
