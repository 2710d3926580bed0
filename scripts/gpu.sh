#!/bin/bash
# One parameterised GPU runner (replaces the round-1..3 one-off gpu_*.sh scripts).
#
#   bash scripts/gpu.sh <outdir-name> <step> [<step> ...]
#
# steps (each runs under its own time limit; the first failure ends the call):
#   tests        pytest -m gpu (whole suite, one process)
#   tests:EXPR   pytest -m gpu -k EXPR
#   smoke        __graft_entry__.smoke()
#   bench        driver window x2 (python bench.py --steps 20 --warmup 5)
#   bench100     100 timed steps, RPC under load
#   b1           batch-1 bench (400 steps)
#   b1lat        batch-1 bench at lag 0 (each step's records collected in the step: latency mode)
#   b1lag1       batch-1 bench at lag 1
#   cfg4         DeepLabv3-ResNet50 1025^2 int8 B=8 (60 steps) and bf16
#   cfg5         4 camera streams x 8 frames (batched step)
#   cfg5p        the same with one engine + HIP stream + hipGraph per camera stream
#   prof         sequential kernel trace of the B=32 step -> layer_times.txt
#   profb1       sequential kernel trace of the B=1 step -> b1_layer_times.txt
#   prof0        the B=32 trace at lag 0 (post-processing not overlapping the next step)
#   profc4       config-4 (ResNet-50 1025^2 int8, B=8) kernel trace -> c4_roofline.txt
#   pmc          3 SQ counter passes over the sequential B=32 step -> pmc_summary.txt
#   pmck         the same passes per kernel name + grid (model from BENCH_ARGS) -> kernel_pmc.txt
#   race         concurrent-plan determinism check (scripts/debug_race.py)
#   share8 / share:N  the dpN bench path with N ranks sharing this one GPU (SSA_SHARE_GPU=1, gloo;
#                completes end to end -- its throughput is not a scaling number)
#   postab       post-processing harness (tools/bin/post_bench), strips vs 32^2 / 64^2 tile accumulation
#   postvar      every tools/bin/pb_* variant (scripts/post_variants.sh) on the bench model's own label
#                maps + the synthetic kinds (POST_DBG_LIST: SSA_POST_DBG values; STAGEWISE=1: per launch)
#   postpmc      3 SQ counter passes over tools/bin/pb_prod on the bench model's label maps -> post_pmc.txt
#   posttrace    post_bench (4 map kinds incl. the fallback-path lattice) under a kernel trace
#   repro        packed-f32 co-residence reproducer, both builds (csrc/tools/packed_f32_repro.hip)
#   tunec4       autotune config 4 (ResNet-50 1025^2 B=8, int8 and bf16) into $O/tune.json
#   usetune      copy $O/tune.json over assets/tune_mi355x.json in the box's tree (then commit it here)
#   upbench      upsample+argmax variant microbench (scripts/bench_upsample.py)
#   retune:LIST  re-time the named choices (comma list) at B = ${TUNE_B:-32} on top of the committed
#                picks -> $O/tune.json (copy into assets/tune_mi355x.json to commit)
#   retuneall:B  re-time EVERY choice of the B-frame plan (SSA_RETUNE=1) -> $O/tune.json
#   py:SCRIPT    python SCRIPT (args in PY_ARGS)
# Extra env: BENCH_ARGS is appended to every bench.py call.
set -o pipefail
cd "$(dirname "$0")/.."
REPO=$PWD
export SSA_NO_AUTOBUILD=1
# the trace steps run from /tmp: a relative tune file must not silently vanish there
[ -n "$SSA_TUNE_FILE" ] && export SSA_TUNE_FILE=$(realpath -m "$SSA_TUNE_FILE")
O=gpurun_out/${1:?outdir}
shift
mkdir -p $O
PMC_SETS=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH"
)

trace() {  # trace <name> <bench args...>: sequential-model kernel trace + layer table
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && SSA_SLOT_PARALLEL=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d $REPO/$O/$name -o run --output-format csv -- python3 $REPO/bench.py "$@" --lag ${TRACE_LAG:-1} --rpc 0 $BENCH_ARGS \
    > $REPO/$O/$name.log 2>&1) || { echo "trace $name failed"; tail -5 $O/$name.log; return 1; }
  python3 scripts/layer_times.py $(ls $O/$name/*/run_kernel_trace.csv 2>/dev/null || ls $O/$name/run_kernel_trace.csv) \
    > $O/${name}_layer_times.txt && tail -45 $O/${name}_layer_times.txt
}

bench() {  # bench <tag> <seconds> <args...>
  local tag=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" $BENCH_ARGS > $O/bench_$tag.json 2> $O/bench_$tag.err \
    || { echo "bench $tag failed rc=$?"; grep -v "^frame" $O/bench_$tag.err | tail -8; return 1; }
  cut -c1-400 $O/bench_$tag.json
}

for step in "$@"; do
  echo "== $step"
  case $step in
    tests)   timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
               > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }; tail -2 $O/pytest.txt ;;
    tests:*) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
               -k "${step#tests:}" > $O/pytest_k.txt 2>&1 || { tail -30 $O/pytest_k.txt; exit 1; }; tail -5 $O/pytest_k.txt ;;
    smoke)   timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
               || { tail -20 $O/smoke.txt; exit 1; }; tail -3 $O/smoke.txt ;;
    bench)   bench d1 300 --steps 20 --warmup 5 && bench d2 300 --steps 20 --warmup 5 || exit 2 ;;
    bench100) bench s100 300 --steps 100 --warmup 10 || exit 2 ;;
    b1)      bench b1 300 --batch 1 --steps 400 --warmup 50 --rpc 0 || exit 2 ;;
    b1lat)   bench b1lat 300 --batch 1 --lag 0 --steps 400 --warmup 50 --rpc 0 || exit 2 ;;
    b1lag1)  bench b1lag1 300 --batch 1 --lag 1 --steps 400 --warmup 50 --rpc 0 || exit 2 ;;
    cfg4)    bench c4i8 400 --arch resnet50 --input_size 1025 --camera 2048x1024 --batch 8 --dtype int8 --steps 60 --warmup 5 --rpc 0 \
               && bench c4bf 400 --arch resnet50 --input_size 1025 --camera 2048x1024 --batch 8 --steps 60 --warmup 5 --rpc 0 || exit 2 ;;
    cfg5)    bench c5 300 --streams 4 --batch 32 --steps 100 --warmup 10 --rpc 0 || exit 2 ;;
    cfg5p)   bench c5p 400 --streams 4 --batch 32 --per_stream_graphs --steps 100 --warmup 10 --rpc 0 || exit 2 ;;
    prof)    trace seq --steps 5 --warmup 2 || exit 3 ;;
    profb1)  trace b1seq --batch 1 --steps 20 --warmup 5 || exit 3 ;;
    prof0)   TRACE_LAG=0 trace seq0 --steps 5 --warmup 2 || exit 3 ;;
    profc4)  trace c4seq --arch resnet50 --input_size 1025 --camera 2048x1024 --batch 8 --dtype int8 --steps 5 --warmup 2 || exit 3
             python3 scripts/roofline_int8.py $(ls $O/c4seq/*/run_kernel_trace.csv 2>/dev/null || ls $O/c4seq/run_kernel_trace.csv) 8 \
               > $O/c4_roofline.txt && head -3 $O/c4_roofline.txt && tail -3 $O/c4_roofline.txt ;;
    pmc)     i=0
             for set in "${PMC_SETS[@]}"; do
               i=$((i+1))
               (cd /tmp && export TMPDIR=/tmp && SSA_SLOT_PARALLEL=0 timeout -s KILL 180 rocprofv3 --pmc $set \
                 -d $REPO/$O/pmc$i -o run --output-format csv -- python3 $REPO/bench.py --steps 3 --warmup 1 --lag 1 --rpc 0 $BENCH_ARGS \
                 > $REPO/$O/pmc$i.log 2>&1) || { echo "pmc set $i failed"; tail -5 $O/pmc$i.log; exit 4; }
             done
             python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 $O/pmc3 > $O/pmc_summary.txt 2>&1; head -60 $O/pmc_summary.txt ;;
    pmck)    i=0  # the same 3 passes, summarised per kernel name (pmc_kernels.py); model picked by BENCH_ARGS
             for set in "${PMC_SETS[@]}"; do
               i=$((i+1))
               (cd /tmp && export TMPDIR=/tmp && SSA_SLOT_PARALLEL=0 timeout -s KILL 240 rocprofv3 --pmc $set \
                 -d $REPO/$O/kpmc$i -o run --output-format csv -- python3 $REPO/bench.py --steps 3 --warmup 1 --lag 1 --rpc 0 $BENCH_ARGS \
                 > $REPO/$O/kpmc$i.log 2>&1) || { echo "pmc set $i failed"; tail -5 $O/kpmc$i.log; exit 4; }
             done
             PMC_BY_GRID=1 python3 scripts/pmc_kernels.py $O/kpmc1 $O/kpmc2 $O/kpmc3 > $O/kernel_pmc.txt 2>&1; rm -rf $O/kpmc?; grep -c "^==" $O/kernel_pmc.txt ;;
    race)    timeout -k 10 600 python scripts/debug_race.py $RACE_ARGS > $O/race.txt 2>&1 || { tail -20 $O/race.txt; exit 5; }; tail -5 $O/race.txt ;;
    share8|share:*) n=${step#share}; n=${n#:}
             SSA_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
               --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus $n --steps 10 --warmup 3 --rpc 300 $BENCH_ARGS \
               > $O/share$n.json 2> $O/share$n.err || { grep -v "^\[Gloo\]" $O/share$n.err | tail -30; exit 5; }
             cut -c1-600 $O/share$n.json ;;
    postab)  for m in 0 1 2; do SSA_POST_ACCUM=$m timeout -k 10 120 tools/bin/post_bench 50 > $O/post_accum$m.txt 2>&1 \
               || { tail -5 $O/post_accum$m.txt; exit 7; }; echo "accum=$m"; cat $O/post_accum$m.txt; done ;;
    postvar) [ -f /tmp/ssa_maps.bin ] || timeout -k 10 300 python scripts/label_stats.py /tmp/ssa_maps.bin > $O/label_stats.txt 2>&1 \
               || { tail -5 $O/label_stats.txt; exit 7; }
             for bin in tools/bin/pb_*; do for d in ${POST_DBG_LIST:-0}; do
               env SSA_POST_DBG=$d ${STAGEWISE:+SSA_POST_STAGEWISE=1} timeout -k 10 180 $bin ${POST_REPS:-30} /tmp/ssa_maps.bin \
                 > $O/$(basename $bin)_d$d.txt 2>&1 || { tail -5 $O/$(basename $bin)_d$d.txt; exit 7; }
               echo "== $bin dbg=$d"; cat $O/$(basename $bin)_d$d.txt; done; done ;;
    postpmc) [ -f /tmp/ssa_maps.bin ] || timeout -k 10 300 python scripts/label_stats.py /tmp/ssa_maps.bin > $O/label_stats.txt 2>&1 \
               || { tail -5 $O/label_stats.txt; exit 7; }
             i=0
             for set in "${PMC_SETS[@]}"; do
               i=$((i+1))
               (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $set \
                 -d $REPO/$O/ppmc$i -o run --output-format csv -- $REPO/tools/bin/pb_prod 5 /tmp/ssa_maps.bin 1 \
                 > $REPO/$O/ppmc$i.log 2>&1) || { echo "pmc set $i failed"; tail -5 $O/ppmc$i.log; exit 4; }
             done
             python3 scripts/pmc_kernels.py $O/ppmc1 $O/ppmc2 $O/ppmc3 > $O/post_pmc.txt 2>&1; cat $O/post_pmc.txt ;;
    posttrace) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
               -d $REPO/$O/posttrace -o run --output-format csv -- $REPO/tools/bin/post_bench 20 \
               > $REPO/$O/posttrace.log 2>&1) || { tail -5 $O/posttrace.log; exit 7; }
             grep -E "us/call|workspace" $O/posttrace.log
             head -12 $(ls $O/posttrace/*/run_kernel_stats.csv $O/posttrace/run_kernel_stats.csv 2>/dev/null | head -1) | cut -d, -f1-8 ;;
    repro)   for b in repro_pk repro_nopk; do timeout -k 10 300 tools/bin/$b ${REPRO_REPS:-400} > $O/$b.txt 2>&1 \
               || { tail -5 $O/$b.txt; exit 7; }; cat $O/$b.txt; done ;;
    tunec4)  [ -f $O/tune.json ] || cp assets/tune_mi355x.json $O/tune.json  # config-4 plans (int8, bf16) -> $O/tune.json
             for dt in int8 bf16; do
               SSA_TUNE_FILE=$O/tune.json SSA_LOG_AUTOTUNE=1 timeout -k 10 600 python bench.py --arch resnet50 --input_size 1025 \
                 --camera 2048x1024 --batch 8 --dtype $dt --steps 5 --warmup 2 --rpc 0 > $O/tunec4_$dt.json 2> $O/tunec4_$dt.err \
                 || { tail -20 $O/tunec4_$dt.err; exit 8; }
             done; python -c "import json; d=json.load(open('$O/tune.json')); print(sorted(d))" ;;
    usetune) cp $O/tune.json assets/tune_mi355x.json && echo "box tree now runs $O/tune.json" ;;
    upbench) timeout -k 10 120 python scripts/bench_upsample.py > $O/upsample.txt 2>&1 || { tail -5 $O/upsample.txt; exit 9; }
             cat $O/upsample.txt ;;
    retune:*) [ -f $O/tune.json ] || cp assets/tune_mi355x.json $O/tune.json
             SSA_TUNE_FILE=$O/tune.json SSA_RETUNE_ONLY=${step#retune:} SSA_LOG_AUTOTUNE=1 \
               timeout -k 10 600 python bench.py --batch ${TUNE_B:-32} --steps 5 --warmup 2 --rpc 0 $BENCH_ARGS \
               > $O/retune_b${TUNE_B:-32}.json 2> $O/retune_b${TUNE_B:-32}.err || { tail -20 $O/retune_b${TUNE_B:-32}.err; exit 8; }
             grep "autotune" $O/retune_b${TUNE_B:-32}.err | grep -v "picks from" | cut -c1-1500 ;;
    retuneall:*) [ -f $O/tune.json ] || cp assets/tune_mi355x.json $O/tune.json
             b=${step#retuneall:}
             SSA_TUNE_FILE=$O/tune.json SSA_RETUNE=1 SSA_LOG_AUTOTUNE=1 \
               timeout -k 10 600 python bench.py --batch $b --steps 5 --warmup 2 --rpc 0 $BENCH_ARGS \
               > $O/retuneall_b$b.json 2> $O/retuneall_b$b.err || { tail -20 $O/retuneall_b$b.err; exit 8; }
             grep "autotune" $O/retuneall_b$b.err | grep -v "picks from" | cut -c1-300 ;;
    py:*)    timeout -k 10 ${PY_TIMEOUT:-600} python -u ${step#py:} $PY_ARGS > $O/$(basename ${step#py:} .py).txt 2>&1 \
               || { tail -30 $O/$(basename ${step#py:} .py).txt; exit 6; }; tail -${PY_TAIL:-40} $O/$(basename ${step#py:} .py).txt ;;
    *)       echo "unknown step $step"; exit 9 ;;
  esac
done
echo "== all steps ok"
