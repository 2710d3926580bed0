"""DeepLabv3 head (ASPP), full models and the torch reference forward.

Reference behaviour being replaced: ``engine.run_inference`` on the Edge-TPU
DeepLabv3-MobileNetV2 graph returns an H x W label map with the ArgMax already
in-graph (``sem_seg_server.py:162-163``). Our ``DeepLabV3.segment`` reproduces that
contract: normalised input -> logits at output stride -> bilinear upsample
(align_corners=True, as TF ``resize_bilinear`` in DeepLab) -> per-pixel argmax.

ASPP variants:
  * ``full``   : 1x1 + three 3x3 atrous branches (rates 6/12/18) + image pooling
                 (north-star config, 5.36 GMAC/frame at 513^2 for MNv2).
  * ``mobile`` : 1x1 + image pooling only (the TF mobile DeepLab head,
                 2.74 GMAC/frame).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from .layers import ConvBNAct, calibrate_bn, init_random
from .mobilenetv2 import MobileNetV2Backbone
from .resnet import ResNet50Backbone


class ASPP(nn.Module):
    def __init__(self, cin: int, cout: int = 256, rates: Sequence[int] = (6, 12, 18),
                 image_pool: bool = True):
        super().__init__()
        self.rates = tuple(rates)
        self.b0 = ConvBNAct(cin, cout, 1, act="relu")
        self.atrous = nn.ModuleList(ConvBNAct(cin, cout, 3, 1, r, act="relu") for r in self.rates)
        self.pool = ConvBNAct(cin, cout, 1, act="relu") if image_pool else None
        nb = 1 + len(self.rates) + (1 if image_pool else 0)
        self.project = ConvBNAct(nb * cout, cout, 1, act="relu")
        self.cout = cout

    def forward(self, x):
        outs = [self.b0(x)] + [b(x) for b in self.atrous]
        if self.pool is not None:
            p = self.pool(F.adaptive_avg_pool2d(x, 1))
            outs.append(p.expand(-1, -1, x.shape[2], x.shape[3]))
        return self.project(torch.cat(outs, 1))


class DeepLabV3(nn.Module):
    def __init__(self, backbone: nn.Module, num_classes: int, aspp: str = "full",
                 aspp_channels: int = 256):
        super().__init__()
        self.backbone = backbone
        rates = (6, 12, 18) if aspp == "full" else ()
        if backbone.output_stride == 8:
            rates = tuple(2 * r for r in rates)
        self.aspp = ASPP(backbone.out_channels, aspp_channels, rates, image_pool=True)
        self.logits = ConvBNAct(aspp_channels, num_classes, 1, act=None, bias_only=True)
        self.num_classes = num_classes
        self.aspp_kind = aspp

    def forward(self, x):
        """x: normalised NCHW float -> logits at output stride (N, K, h, w)."""
        return self.logits(self.aspp(self.backbone(x)))

    @torch.no_grad()
    def segment(self, x: torch.Tensor, out_hw=None) -> torch.Tensor:
        """x: normalised NCHW -> uint8 label map (N, H, W) at input resolution."""
        logits = self.forward(x).float()
        H, W = out_hw or x.shape[-2:]
        up = F.interpolate(logits, size=(H, W), mode="bilinear", align_corners=True)
        return up.argmax(1).to(torch.uint8)


def build_model(arch: str = "mnv2", num_classes: int = 21, width_mult: float = 1.0,
                output_stride: int = 16, aspp: str = "full", seed: int = 0,
                calibrate_hw: Optional[int] = 129, multi_grid=(1, 2, 4),
                scene_prior: bool = True, calib_input: Optional[torch.Tensor] = None,
                calib_device: Optional[torch.device] = None) -> DeepLabV3:
    """Random-init DeepLabv3 of the named architecture.

    ``calibrate_hw``: side of the synthetic batch used to set BN statistics
    (None to skip); ``calib_input`` (normalised NCHW) replaces that batch, e.g.
    letterboxed camera frames at the deployment resolution: BN statistics and the
    logits prior calibrated on tiny maps do not transfer to 33x33 ones.
    Calibration is deterministic for a given seed.
    """
    if arch == "mnv2":
        bb = MobileNetV2Backbone(width_mult, output_stride)
    elif arch == "resnet50":
        bb = ResNet50Backbone(output_stride, multi_grid)
    else:
        raise ValueError(f"unknown arch {arch!r}")
    model = DeepLabV3(bb, num_classes, aspp)
    init_random(model, seed)
    if calibrate_hw or calib_input is not None:
        if calib_input is not None:
            x = calib_input
        else:
            g = torch.Generator().manual_seed(seed + 1)
            x = synthetic_normalized(2, calibrate_hw, calibrate_hw, g)
        if calib_device is not None:  # fp32 calibration forwards on the GPU, weights back on the host
            model.to(calib_device)
            x = x.to(calib_device)
        calibrate_bn(model, x)
        if scene_prior:
            calibrate_logits(model, x, scene_class_prior(num_classes).to(x.device))
        model.cpu()
    return model.eval()


def scene_class_prior(num_classes: int) -> torch.Tensor:
    """Target pixel share per class for the random-init model's label maps.

    A random-init network collapses to one or two classes (>99 % of pixels), so
    the mask/contour stage would see an empty mask and the benchmark would skip
    the work a deployed server does. The prior makes the classes that survive
    the reference's palette->gray>127 mask (``sem_seg_server.py:77-85``; PASCAL:
    car, person) cover ~35 % of the pixels, background 30 %, the rest evenly.
    """
    from ..labels import GRAY_SHIFT, GRAY_W_B, GRAY_W_G, GRAY_W_R, colormap_for
    cmap = colormap_for("pascal" if num_classes == 21 else "cityscapes")[:num_classes]
    gray = (cmap[:, 0] * GRAY_W_B + cmap[:, 1] * GRAY_W_G + cmap[:, 2] * GRAY_W_R
            + (1 << (GRAY_SHIFT - 1))) >> GRAY_SHIFT
    fg = torch.as_tensor(gray > 127)
    prior = torch.zeros(num_classes)
    prior[fg] = 0.35 / max(int(fg.sum()), 1)
    rest = ~fg
    rest[0] = False
    prior[rest] = 0.35 / max(int(rest.sum()), 1)
    prior[0] += 0.30
    return prior / prior.sum()


@torch.no_grad()
def calibrate_logits(model: "DeepLabV3", x: torch.Tensor, prior: torch.Tensor,
                     iters: int = 40) -> None:
    """Shift the logits-layer bias until the argmax class shares match ``prior``
    (fixed-point iteration b += 0.5 * log(prior / share) on cached features)."""
    was_training = model.training
    model.eval()
    feats = model.aspp(model.backbone(x))
    H, W = x.shape[-2:]
    bias = model.logits.conv.bias
    for _ in range(iters):
        up = F.interpolate(model.logits(feats), size=(H, W), mode="bilinear", align_corners=True)
        share = torch.bincount(up.argmax(1).flatten(), minlength=model.num_classes).float()
        share = share / share.sum()
        bias += 0.5 * (torch.log(prior + 1e-6) - torch.log(share + 1e-3)).clamp(-2, 2)
    model.train(was_training)


def synthetic_normalized(n: int, h: int, w: int, g: Optional[torch.Generator] = None) -> torch.Tensor:
    """Smooth random images in [-1, 1] (blocky, so the argmax map has regions)."""
    g = g or torch.Generator().manual_seed(0)
    coarse = torch.rand((n, 3, max(h // 16, 2), max(w // 16, 2)), generator=g)
    img = F.interpolate(coarse, size=(h, w), mode="bilinear", align_corners=False)
    img = img + 0.1 * torch.randn((n, 3, h, w), generator=g)
    return (img.clamp(0, 1) * 2 - 1).contiguous()


def count_macs(model: DeepLabV3, h: int, w: int) -> int:
    """Multiply-accumulates per frame (convs only), via forward hooks."""
    macs = 0

    def hook(m, inp, out):
        nonlocal macs
        k = m.kernel_size[0] * m.kernel_size[1]
        macs += out.numel() // out.shape[0] * k * (m.in_channels // m.groups)

    hs = [m.register_forward_hook(hook) for m in model.modules() if isinstance(m, nn.Conv2d)]
    with torch.no_grad():
        model(torch.zeros(1, 3, h, w))
    for hd in hs:
        hd.remove()
    return macs
