# round-6 GPU bundle 13: ASPP image pooling -- 32 GAP slices with four loads in flight per
# lane, unrolled pool slices -- full GPU tier, headline, batch 1, both step traces
bash scripts/gpu.sh r8r tests smoke bench prof b1 profb1
