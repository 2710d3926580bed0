# round-6 GPU bundle 18: int8 LDS-DMA GEMM with 64-byte K rows per stage (half the LDS, three
# workgroups per CU) -- int8 kernel tests, full config-4 int8 retune, config-4 benches
bash scripts/gpu.sh r8w "tests:conv_i8" || exit 1
BENCH_ARGS="--arch resnet50 --input_size 1025 --camera 2048x1024 --dtype int8" TUNE_B=8 bash scripts/gpu.sh r8w retuneall:8 || exit 1
bash scripts/gpu.sh r8w usetune cfg4
