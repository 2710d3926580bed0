# round-6 GPU bundle 15: split ASPP pooling with 16 weight loads in flight per thread (two
# launches) -- pooling / model tests, headline, both step traces
bash scripts/gpu.sh r8t "tests:pool or gap or hip_model or headline or graph" bench prof profb1
