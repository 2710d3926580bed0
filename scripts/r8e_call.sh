bash scripts/gpu.sh r8e upbench tests:int8_resnet50_headline tests smoke bench && \
TUNE_B=1 bash scripts/gpu.sh r8e retune:block7,block8,block9,block10,block11,block12,block13,block14,block15,block16,aspp.branches,upsample && \
TUNE_B=32 bash scripts/gpu.sh r8e retune:upsample && \
bash scripts/gpu.sh r8e cfg5 cfg5p cfg4
