# GPU busy fraction of the real (slot-parallel) B = 32 and B = 1 bench runs from kernel
# traces (scripts/busy_fraction.py over the timed steps). Batch-1 depth experiments run
# here before (profiles/r8j_b1_depth_negative.txt): lag 3 5745 fps, lag 3 + 8 HW queues 5554,
# against 6022 at lag 2.
set -e
O=gpurun_out/${OUT:-r8j}; mkdir -p $O; REPO=$PWD
for b in 32 1; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $REPO/$O/sp$b -o run \
     --output-format csv -- python3 $REPO/bench.py --batch $b --steps $((b == 1 ? 600 : 60)) --warmup 10 --rpc 0 \
     > $REPO/$O/sp$b.log 2>&1)
  python3 scripts/busy_fraction.py $(ls $O/sp$b/*/run_kernel_trace.csv 2>/dev/null || ls $O/sp$b/run_kernel_trace.csv) k_records $((b == 1 ? 400 : 40)) > $O/busy_b$b.txt
  echo "== B=$b"; cat $O/busy_b$b.txt
  rm -rf $O/sp$b
done
