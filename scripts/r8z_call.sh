# round-6 GPU bundle 21: stem + block 0 with ReLU6 as [0, 1] clamps folded into the
# conversion / last fma (stem / 6, depthwise bias / 6, projection x 6 in the packing)
bash scripts/gpu.sh r8z "tests:stem or hip_model or headline or graph or golden" bench prof profb1
