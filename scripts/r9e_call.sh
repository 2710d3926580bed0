# round-6 GPU bundle 26: B=32 retune of the front choices and the upsample on the final kernels,
# then the headline on the retuned plan
bash scripts/gpu.sh r9e "retune:stem+block0,block1,block2,block3,block4,block5,block6,upsample" usetune bench prof
