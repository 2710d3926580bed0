# round-6 GPU bundle 8: 32-bit byte offsets against uniform row bases in the slice / band /
# stem_band kernels (global loads and stores off 64-bit VALU address math)
bash scripts/gpu.sh r8m tests bench prof b1
