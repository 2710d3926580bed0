# round-6 GPU bundle 20: final-tree benches -- headline x2, 100 steps, batch 1 at lag 2 / 1,
# config 5 (batched), both step traces
bash scripts/gpu.sh r8y bench bench100 b1 b1lag1 cfg5 prof profb1
