# round-6 GPU bundle 10: 12-wave lattice variant for blocks 14-15 (two depthwise+projection
# waves per SIMD, register-lean depthwise) -- diagnostic, kernel tests, B=32 retune, headline
bash scripts/gpu.sh r8o py:scripts/debug_lattice.py "tests:stream or lattice" retune:block14,block15 usetune bench prof
