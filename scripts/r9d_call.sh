# round-6 GPU bundle 25: per-kernel PMC of the final headline step (3 SQ counter passes)
bash scripts/gpu.sh r9d pmck
