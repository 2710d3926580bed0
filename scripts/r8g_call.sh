# round-6 GPU bundle 2: headline variance (two driver-window runs + 100 steps), batch-1
# latency modes, the lag-0 trace, the host-side profile at batch 1 and the 4-rank rehearsal
bash scripts/gpu.sh r8g bench bench100 b1lat b1lag1 prof0 && \
PY_ARGS="1 2000" bash scripts/gpu.sh r8g py:scripts/profile_host.py && \
bash scripts/gpu.sh r8g share:4 && bash scripts/gpu.sh r8g2 bench
