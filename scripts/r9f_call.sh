# round-6 GPU bundle 27: final-tree long runs -- headline 100 steps, batch 1 at lag 0 / 1,
# config 5 in both forms
bash scripts/gpu.sh r9f bench100 b1lat b1lag1 cfg5 cfg5p
