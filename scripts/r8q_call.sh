# round-6 GPU bundle 12: 3 / 4-stage LDS rings for the int8 LDS-DMA GEMM (config 4) --
# int8 kernel tests, a full config-4 int8 retune (every choice re-timed), the config-4 bench
bash scripts/gpu.sh r8q "tests:conv_i8" || exit 1
BENCH_ARGS="--arch resnet50 --input_size 1025 --camera 2048x1024 --dtype int8" TUNE_B=8 bash scripts/gpu.sh r8q retuneall:8 || exit 1
bash scripts/gpu.sh r8q usetune cfg4
