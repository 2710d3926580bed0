"""Per-layer comparison of the int8 DeepLabv3-ResNet50 plan against the fp32 fake-quant
replay (models/quant.py) at a given shape: for every quantisation point, the fraction of
int8 codes that differ and the largest difference, so a divergence can be located.

  python scripts/int8_layer_diff.py [B] [input] [camW]x[camH] [calib: engine|frames]
"""
import copy
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_server_amd import config as C  # noqa: E402
from semantic_segmentation_server_amd.models import quant as Q  # noqa: E402
from semantic_segmentation_server_amd.ops import reference_ops as R  # noqa: E402
from semantic_segmentation_server_amd.runtime.engine import Engine  # noqa: E402
from semantic_segmentation_server_amd.runtime.sources import SyntheticSource  # noqa: E402


@torch.no_grad()
def fq_points(model, S, x, stem_bf16=False):
    """The fake-quant replay's int8 code tensors (NHWC int) at every quantisation point."""
    bb = model.backbone
    pts = {}

    def conv(layer, inp, s_out=None, res=None, act=None, quant_w=True):
        if quant_w:
            wq, sw, b = Q._qw(layer)
            wf = wq * sw.view(-1, 1, 1, 1)
        else:
            wf, b = layer.fold()
            if stem_bf16:
                wf, inp = wf.to(torch.bfloat16).float(), inp.to(torch.bfloat16).float()
        y = F.conv2d(inp, wf, b, layer.stride, layer.dilation * (layer.k // 2), layer.dilation)
        if res is not None:
            y = y + res
        a = layer.act if act is None else act
        if a == "relu":
            y = torch.relu(y)
        return Q.q(y, s_out) if s_out is not None else y

    def code(name, t, s):
        pts[name] = torch.round(t / s).permute(0, 2, 3, 1).to(torch.int32)

    h = conv(bb.stem, x, S["stem"], quant_w=False)
    code("stem", h, S["stem"])
    h = F.max_pool2d(h, 3, 2, 1)
    code("pool0", h, S["stem"])
    for i, blk in enumerate(bb.blocks):
        idt = h if blk.down is None else conv(blk.down, h, S[f"b{i}.down"])
        if blk.down is not None:
            code(f"r{i}_down", idt, S[f"b{i}.down"])
        t1 = conv(blk.conv1, h, S[f"b{i}.c1"])
        code(f"r{i}_c1", t1, S[f"b{i}.c1"])
        t2 = conv(blk.conv2, t1, S[f"b{i}.c2"])
        code(f"r{i}_c2", t2, S[f"b{i}.c2"])
        h = conv(blk.conv3, t2, S[f"b{i}.out"], res=idt, act="relu")
        code(f"r{i}_out", h, S[f"b{i}.out"])
    return pts


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 1025
    cw, ch = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "2048x1024").split("x"))
    calib = sys.argv[4] if len(sys.argv) > 4 else "engine"
    dev = torch.device("cuda", 0)
    cfg = C.Config(arch="resnet50", dtype="int8", input_size=S, batch=B, backend="hip", graph=False,
                   num_classes=19, dataset="cityscapes", camera_width=cw, camera_height=ch)
    eng = Engine(cfg, dev)
    eng.set_camera(cw, ch)
    f, _, _ = SyntheticSource(cw, ch, pool=4, seed=21).read_batch(B)
    frames = torch.from_numpy(np.ascontiguousarray(f)).to(dev)
    x = R.preprocess(frames.cpu(), eng.lut_x.cpu(), eng.lut_y.cpu()).to(dev)
    m32 = copy.deepcopy(eng.model).float().to(dev)
    hm = eng._hip_model
    if calib == "frames":
        from semantic_segmentation_server_amd.models.hip_int8 import HipDeepLabInt8
        hm = HipDeepLabInt8(eng.model, dev, cfg, scales=Q.calibrate(m32, x))
    logits = hm.logits(frames, eng.lut_x, eng.lut_y).float()
    torch.cuda.synchronize()
    bufs = hm._plans[(B, ch, cw)][1]
    sb = hm.choices.get("stem", "fp32") != "fp32"
    pts = fq_points(m32, hm.scales, x, stem_bf16=sb)
    print(f"B={B} S={S} cam={cw}x{ch} calib={calib} stem={hm.choices.get('stem')}")
    for name, ref in pts.items():
        got = bufs[name].to(torch.int32)
        d = (got - ref).abs()
        sat = (ref.abs() >= 127).float().mean().item()
        print(f"{name:10s} mismatch {(d > 0).float().mean().item():.5f} max {int(d.max())} "
              f"saturated {sat:.4f}", flush=True)
    ref = Q.fake_quant_forward(m32, hm.scales, x, stem_bf16=sb).float()
    got = logits.permute(0, 3, 1, 2)
    print(f"logits rel err vs fake-quant {((got - ref).norm() / ref.norm()).item():.4f}")


if __name__ == "__main__":
    main()
