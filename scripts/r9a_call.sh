# round-6 GPU bundle 22: upsample + argmax specialised on the exact class count (21 / 19)
# -- upsample tests, variant microbench, headline + step trace, config 4
bash scripts/gpu.sh r9a "tests:upsample" upbench bench prof cfg4
