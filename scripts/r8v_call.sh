# round-6 GPU bundle 17: config-4 int8 step trace on the current tree (roofline table)
bash scripts/gpu.sh r8v profc4
