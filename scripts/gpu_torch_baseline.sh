set -o pipefail
cd /root/repo
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/g1_info.txt 2>&1
timeout -k 10 300 python bench.py --backend torch --contour_mode none --steps 10 --warmup 3 --rpc 0 > gpurun_out/g1_torch_graph.json 2> gpurun_out/g1_torch_graph.err && \
timeout -k 10 300 python bench.py --backend torch --contour_mode none --steps 10 --warmup 3 --rpc 0 --no-graph > gpurun_out/g1_torch_eager.json 2> gpurun_out/g1_torch_eager.err && \
timeout -k 10 300 python bench.py --backend torch --contour_mode none --steps 10 --warmup 3 --rpc 0 --batch 1 > gpurun_out/g1_torch_b1.json 2> gpurun_out/g1_torch_b1.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/g1_prof -o run --output-format csv -- python3 /root/repo/bench.py --backend torch --contour_mode none --steps 5 --warmup 2 --rpc 0 > /root/repo/gpurun_out/g1_prof.log 2>&1
