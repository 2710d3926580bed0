# round-6 GPU bundle 11: batch-1 retune of blocks 14-16 with the lattice spans offered
# (S = 16 / 32, hidden split), then the batch-1 bench and step trace on the retuned plan
TUNE_B=1 bash scripts/gpu.sh r8p retune:block14,block15,block16 usetune b1 b1lag1 profb1
