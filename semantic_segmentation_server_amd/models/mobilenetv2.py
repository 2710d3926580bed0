"""MobileNetV2 backbone with output-stride control (DeepLabv3 feature extractor).

The reference's model is ``deeplabv3_mnv2_pascal_quant_edgetpu.tflite``
(``sem_seg_server.py:238``): DeepLabv3 on MobileNetV2, depth multiplier 1.0,
output stride 16. We rebuild the architecture: stem 3x3/2 -> 17 inverted
residual blocks, with the atrous trick of TF-slim's ``mobilenet`` when the
running stride reaches ``output_stride``: the unit that would exceed it gets
stride 1 and the *following* units get dilation ``rate *= stride``. Features are
the 320-channel output of the last block (the 1280-channel head conv is not
used by DeepLab).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.nn as nn

from .layers import ConvBNAct, make_divisible

# (expansion t, channels c, repeats n, first stride s)
MNV2_SETTINGS = [
    (1, 16, 1, 1),
    (6, 24, 2, 2),
    (6, 32, 3, 2),
    (6, 64, 4, 2),
    (6, 96, 3, 1),
    (6, 160, 3, 2),
    (6, 320, 1, 1),
]


@dataclass
class IRSpec:
    cin: int
    cout: int
    expand: int
    stride: int
    dilation: int

    @property
    def hidden(self) -> int:
        return self.cin * self.expand

    @property
    def residual(self) -> bool:
        return self.stride == 1 and self.cin == self.cout


class InvertedResidual(nn.Module):
    def __init__(self, spec: IRSpec):
        super().__init__()
        self.spec = spec
        hid = spec.hidden
        self.expand = ConvBNAct(spec.cin, hid, 1, act="relu6") if spec.expand != 1 else None
        self.dw = ConvBNAct(hid, hid, 3, spec.stride, spec.dilation, groups=hid, act="relu6")
        self.project = ConvBNAct(hid, spec.cout, 1, act=None)

    def forward(self, x):
        y = x
        if self.expand is not None:
            y = self.expand(y)
        y = self.project(self.dw(y))
        return x + y if self.spec.residual else y


def mnv2_block_specs(width_mult: float = 1.0, output_stride: int = 16) -> (int, List[IRSpec]):
    stem_c = make_divisible(32 * width_mult, 8)
    specs: List[IRSpec] = []
    cur_stride, rate = 2, 1
    cin = stem_c
    for t, c, n, s in MNV2_SETTINGS:
        cout = make_divisible(c * width_mult, 8)
        for i in range(n):
            stride = s if i == 0 else 1
            if output_stride is not None and cur_stride * stride > output_stride:
                layer_stride, layer_rate = 1, rate
                rate *= stride
            else:
                layer_stride, layer_rate = stride, rate if stride == 1 else 1
                cur_stride *= stride
            specs.append(IRSpec(cin, cout, t, layer_stride, layer_rate))
            cin = cout
    return stem_c, specs


class MobileNetV2Backbone(nn.Module):
    def __init__(self, width_mult: float = 1.0, output_stride: int = 16):
        super().__init__()
        stem_c, specs = mnv2_block_specs(width_mult, output_stride)
        self.stem = ConvBNAct(3, stem_c, 3, 2, act="relu6")
        self.blocks = nn.ModuleList(InvertedResidual(s) for s in specs)
        self.out_channels = specs[-1].cout
        self.output_stride = output_stride

    def forward(self, x):
        x = self.stem(x)
        for b in self.blocks:
            x = b(x)
        return x
