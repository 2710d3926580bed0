# round-6 GPU bundle: tests, retunes (batch 1 tail with the hoisted in-launch combines; the
# upsample variants at B = 32), then the benches and traces on the retuned plans
bash scripts/gpu.sh r8f tests smoke && \
TUNE_B=1 bash scripts/gpu.sh r8f retune:block7,block8,block9,block10,block11,block12,block13,block14,block15,block16,aspp.branches,upsample && \
TUNE_B=32 bash scripts/gpu.sh r8f retune:upsample usetune && \
bash scripts/gpu.sh r8f bench b1 cfg5 cfg5p cfg4 prof profb1
