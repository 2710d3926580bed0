# round-6 GPU bundle 7: MFMA results in VGPRs for every source + the stem_band ring offsets
# -- full GPU tier, smoke, headline / batch-1 / config-4 benches, step traces
bash scripts/gpu.sh r8l tests smoke bench b1 cfg4 prof profb1
