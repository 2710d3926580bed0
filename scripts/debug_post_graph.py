"""Isolate the post-processing kernels: eager (no sync) vs graph replay per batch size."""
import sys
import numpy as np
import torch
from semantic_segmentation_server_amd.labels import pascal_colormap
from semantic_segmentation_server_amd.postprocess.device import DevicePostprocess
from semantic_segmentation_server_amd.postprocess.synthetic import random_label_map

mode = sys.argv[1]
B = int(sys.argv[2])
src = sys.argv[3] if len(sys.argv) > 3 else "planted"
H = W = 513
rng = np.random.default_rng(0)
if src == "planted":
    maps = np.stack([random_label_map(rng, H, W) for _ in range(B)])
else:  # near-constant maps like a random-init model produces
    maps = np.full((B, H, W), 4, np.uint8)
    maps[:, 200:260, 100:400] = 6
dev = torch.device("cuda")
lab = torch.from_numpy(maps).to(dev)
post = DevicePostprocess(dev, H, W, pascal_colormap(), K=64)
out = post.run(lab, 513, 384, 0.05 * 513 * 513)
torch.cuda.synchronize()
ref = out.clone()
print("eager ok", mode, B, src, int(ref[:, 0].sum().item()), flush=True)
if mode == "graph":
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        post.run(lab, 513, 384, 0.05 * 513 * 513)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        o = post.run(lab, 513, 384, 0.05 * 513 * 513)
    for i in range(3):
        g.replay()
        torch.cuda.synchronize()
        print("replay", i, "equal", torch.equal(o, ref), flush=True)
