set -o pipefail
export SSA_NO_AUTOBUILD=1
mkdir -p gpurun_out/b1ab
for i in 1 2; do
for t in assets/tune_mi355x.json candidate picks; do
  SSA_TUNE_FILE=$PWD/$t timeout -k 10 200 python bench.py --batch 1 --steps 400 --warmup 50 --rpc 0 > gpurun_out/b1ab/b1_$i.json 2> gpurun_out/b1ab/b1_$i.err || exit 1
  echo "$t $(python -c "import json;d=json.load(open('gpurun_out/b1ab/b1_$i.json'));print(d['ms_per_step'])")"
done; done
