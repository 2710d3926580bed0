# round-6 GPU bundle 16: depthwise VALU of the stream kernel's projection waves at raised
# issue priority (dwproj_chunk: MODE 0 / 4 blocks 14-15) -- stream tests, headline trace x2
bash scripts/gpu.sh r8u "tests:stream" bench prof && cp gpurun_out/r8u/seq_layer_times.txt gpurun_out/r8u/seq_layer_times_1.txt && bash scripts/gpu.sh r8u prof
