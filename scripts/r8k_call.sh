# round-6 GPU bundle 6: letterbox pre-pass + dense stems (goldens; stem retunes at the
# config-4 shape, int8 and bf16; config-4 benches) and the GPU busy fraction of the
# headline / batch-1 runs
bash scripts/gpu.sh r8k tests:stem && \
BENCH_ARGS="--arch resnet50 --input_size 1025 --camera 2048x1024 --dtype int8" TUNE_B=8 \
  bash scripts/gpu.sh r8k retune:stem && \
BENCH_ARGS="--arch resnet50 --input_size 1025 --camera 2048x1024" TUNE_B=8 \
  bash scripts/gpu.sh r8k retune:stem usetune && \
bash scripts/gpu.sh r8k cfg4 tests:int8_resnet50_headline && OUT=r8k bash scripts/gpu_busy.sh
