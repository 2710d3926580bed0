# round-6 GPU bundle 23: final tree -- full GPU tier, smoke, headline, batch 1, config 4
bash scripts/gpu.sh r9b tests smoke bench b1 cfg4
