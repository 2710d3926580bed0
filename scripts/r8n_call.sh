# round-6 GPU bundle 9: lattice spans for the dilation-2 blocks 14-16 (halo +- 1 lattice row,
# 3 expansion rounds instead of 5) -- kernel tests, B=32 retune of blocks 14-16, headline
bash scripts/gpu.sh r8n py:scripts/debug_lattice.py "tests:stream or lattice" retune:block14,block15,block16 usetune bench prof
