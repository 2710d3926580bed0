# round-6 GPU bundle 5: GPU busy fraction of the real (slot-parallel) B = 32 and B = 1 runs
# from kernel traces, and two batch-1 depth experiments (lag 3; lag 3 with 8 HW queues)
set -e
O=gpurun_out/r8j; mkdir -p $O; REPO=$PWD
for b in 32 1; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/$O/sp$b -o run \
     --output-format csv -- python3 $REPO/bench.py --batch $b --steps $((b == 1 ? 600 : 60)) --warmup 10 --rpc 0 \
     > $REPO/$O/sp$b.log 2>&1)
  python3 scripts/busy_fraction.py $(ls $O/sp$b/*/run_kernel_trace.csv 2>/dev/null || ls $O/sp$b/run_kernel_trace.csv) > $O/busy_b$b.txt
  echo "== B=$b"; cat $O/busy_b$b.txt
  rm -rf $O/sp$b
done
SSA_PIPE_LAG=3 bash scripts/gpu.sh r8j_l3 b1
SSA_PIPE_LAG=3 GPU_MAX_HW_QUEUES=8 bash scripts/gpu.sh r8j_q8 b1
