"""Compare device CCL labels (from the post-processing workspace) with scipy."""
import numpy as np
import torch
from semantic_segmentation_server_amd.labels import pascal_colormap
from semantic_segmentation_server_amd.postprocess.components import label_components
from semantic_segmentation_server_amd.postprocess.device import DevicePostprocess
from semantic_segmentation_server_amd.postprocess.reference import palette_mask_numpy
from semantic_segmentation_server_amd.postprocess.synthetic import random_label_map

def al(x): return (x + 255) & ~255
rng = np.random.default_rng(0)
B, h, w, H, W, K, bins = 4, 513, 513, 513, 513, 64, 32
maps = np.zeros((B, H, W), np.uint8)
for i in range(B):
    maps[i] = rng.integers(0, 21, (H, W), dtype=np.uint8)
    maps[i, :h, :w] = random_label_map(rng, h, w, n_blobs=int(rng.integers(1, 8)), noise=float(rng.choice([0.0, 0.01])))
dev = torch.device("cuda")
post = DevicePostprocess(dev, H, W, pascal_colormap(), K=K)
for rep in range(12):
    post.run(torch.from_numpy(maps).to(dev), w, h, 0.05 * 513 * 513)
    torch.cuda.synchronize()
    ws = post._bufs[B][0].cpu().numpy()
    N = H * W
    small = al(16 + K * bins * 4 + K * 4)
    big = al((N + 1) * 4) + al(N) + 4 * al(N * 4) + 4 * al(N * 8)
    for b in range(B):
        base = B * small + b * big
        L = ws[base: base + (N + 1) * 4].view(np.int32)
        mk = ws[base + al((N + 1) * 4): base + al((N + 1) * 4) + N]
        n = h * w
        dev_node = L[1:n + 1].reshape(h, w)
        dev_mask = mk[:n].reshape(h, w)
        ref_mask = palette_mask_numpy(maps[b, :h, :w]) > 0
        node, fg = label_components(ref_mask)
        mm = (dev_mask.astype(bool) != ref_mask).sum()
        bad = np.argwhere(dev_node != node)
        print(f"rep {rep} frame {b}: mask mismatches {mm}, label mismatches {len(bad)}")
        for (y, x) in bad[:8]:
            print("   ", y, x, "dev", dev_node[y, x], "ref", node[y, x], "fg", fg[y, x])
