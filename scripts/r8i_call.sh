# round-6 GPU bundle 4: per-lane-candidate upsample variant -- microbench, goldens, retunes
# at B = 32 / 1 on the bench model's logits, headline bench, per-kernel PMC of the step
bash scripts/gpu.sh r8i upbench tests:upsample && \
TUNE_B=32 bash scripts/gpu.sh r8i retune:upsample && TUNE_B=1 bash scripts/gpu.sh r8i retune:upsample usetune && \
bash scripts/gpu.sh r8i bench b1 pmck
