"""Statistics of the label maps the bench actually feeds the post-processing
(random-init DeepLabv3-MNv2 on synthetic camera frames): class mix, foreground
share, component counts, selected contours per frame."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.postprocess.components import label_components  # noqa: E402
from semantic_segmentation_server_amd.postprocess.reference import palette_mask_numpy  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402


def main():
    B = 32
    eng = Engine(C.Config(backend="hip", batch=B, graph=False), torch.device("cuda", 0))
    eng.set_camera(640, 480)
    src = SyntheticSource(640, 480, seed=1, pool=8)
    frames = torch.from_numpy(src.read_batch(B)[0]).cuda()
    labels, post = eng._step_device(frames)
    full = labels.cpu().numpy()
    if len(sys.argv) > 1:  # raw [B, H, W] uint8 dump for csrc/tools/post_bench.hip
        full.astype(np.uint8).tofile(sys.argv[1])
        print("dumped", full.shape, "to", sys.argv[1])
    lab = full[:, :eng.crop_h, :eng.crop_w]
    rec = post.cpu().numpy()
    print("crop", eng.crop_w, eng.crop_h, "records/frame", rec[:, 0].mean())
    cls, cnt = np.unique(lab, return_counts=True)
    print("classes", dict(zip(cls.tolist(), (cnt / cnt.sum()).round(3).tolist())))
    for i in range(0, B, 4):
        m = palette_mask_numpy(lab[i])
        node, fg = label_components(m)
        nfg = len(np.unique(node[fg])) if fg.any() else 0
        nbg = len(np.unique(node[~fg])) if (~fg).any() else 0
        print(f"frame {i}: fg {m.mean():.3f} records {rec[i, 0]:.0f} fg comps {nfg} bg comps {nbg} "
              f"inside-pixels {(node != 0).mean():.3f}")


if __name__ == "__main__":
    main()
