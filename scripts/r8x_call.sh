# round-6 GPU bundle 19: the int8 ASPP branches on the 64-byte-K-row tiles (sep18) -- retune of
# the ASPP choice on the committed config-4 plan, config-4 benches, full GPU tier + smoke
BENCH_ARGS="--arch resnet50 --input_size 1025 --camera 2048x1024 --dtype int8" TUNE_B=8 bash scripts/gpu.sh r8x retune:aspp_i8 || exit 1
bash scripts/gpu.sh r8x usetune cfg4 tests smoke
