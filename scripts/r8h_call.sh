# round-6 GPU bundle 3: host-path changes (fast stream switches, event rings) -- tests,
# smoke, headline + batch-1 benches, the batch-1 host profile
bash scripts/gpu.sh r8h tests smoke bench b1 b1lag1 && \
PY_ARGS="1 2000" bash scripts/gpu.sh r8h py:scripts/profile_host.py
