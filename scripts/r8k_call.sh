# round-6 GPU bundle 6: letterbox pre-pass + dense int8 stem (goldens, int8 stem retune at the
# config-4 shape, config-4 bench) and the GPU busy fraction of the headline / batch-1 runs
bash scripts/gpu.sh r8k tests:stem && \
BENCH_ARGS="--arch resnet50 --input_size 1025 --camera 2048x1024 --dtype int8" TUNE_B=8 \
  bash scripts/gpu.sh r8k retune:stem usetune && \
bash scripts/gpu.sh r8k cfg4 tests:int8_resnet50_headline && OUT=r8k bash scripts/gpu_busy.sh
