#!/bin/bash
# Builds post_bench variants of csrc/hip/postprocess.hip (CPU side, before a GPU call):
#   bash scripts/post_variants.sh tag:"-DFLAG ..." [tag:"..."] ...
# -> tools/bin/pb_<tag>; scripts/gpu.sh step "postvar" runs every tools/bin/pb_* binary.
set -e
cd "$(dirname "$0")/.."
rm -f tools/bin/pb_*
for spec in "$@"; do
  tag=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc/hip $flags \
    csrc/tools/post_bench.hip csrc/hip/postprocess.hip -o tools/bin/pb_$tag &
done
wait
ls -la tools/bin/pb_*
