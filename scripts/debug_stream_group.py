"""Debug: StreamGroup with bound staging slots and split model / post graphs vs a
single engine on the same frames (records and per-engine label maps)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SSA_FUSED_IR"] = "1"
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.multistream import StreamGroup  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402

cfg = C.Config(input_size=129, batch=4, backend="hip", graph=True)
grp = StreamGroup(cfg, torch.device("cuda"), 2)
one = Engine(cfg, torch.device("cuda"))
for e in (grp, one):
    e.set_camera(200, 150)
f, _, _ = SyntheticSource(200, 150, pool=4).read_batch(4)
d = torch.from_numpy(f).cuda()
l1, p1 = one.run_device(d)
l1, p1 = l1.clone(), p1.clone()
for _ in range(2):
    _, p2 = grp.run_device(d)
torch.cuda.synchronize()
p2 = p2.clone()
print("p1==p2", torch.equal(p1, p2), p1[:, :3].tolist(), p2[:, :3].tolist(), flush=True)
bufs = [torch.empty_like(d) for _ in range(2)]
grp.bind_inputs(bufs, split_post=True)
for it in range(2):
    for si, b in enumerate(bufs):
        b.copy_(d)
        torch.cuda.synchronize()
        _, p3 = grp.run_device(b)
        with torch.cuda.stream(grp.result_stream):
            p3c = p3.clone()
        torch.cuda.synchronize()
        labs = [e._bound_graphs[b.chunk(2)[i].data_ptr()][2] for i, e in enumerate(grp.engines)]
        print(it, si, "p3==p1", torch.equal(p3c, p1), p3c[:, :3].tolist(),
              "labels==one", [torch.equal(lab, l1[2 * i:2 * i + 2]) for i, lab in enumerate(labs)], flush=True)
