"""ResNet-50 backbone with dilation (DeepLabv3-ResNet50, BASELINE config 4).

Not present in the reference (its only model is the Edge-TPU MobileNetV2 tflite,
``sem_seg_server.py:238``); added for the 1025x1025 Cityscapes-19 int8 config of
``BASELINE.json``. ResNet v1.5 bottlenecks (stride on the 3x3); for output stride
16 the last stage uses stride 1 / dilation 2 (DeepLabv3 multi-grid optional),
for output stride 8 stages 3/4 use dilation 2/4.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from .layers import ConvBNAct


class Bottleneck(nn.Module):
    def __init__(self, cin: int, width: int, stride: int, dilation: int, downsample: bool):
        super().__init__()
        cout = width * 4
        self.conv1 = ConvBNAct(cin, width, 1, act="relu")
        self.conv2 = ConvBNAct(width, width, 3, stride, dilation, act="relu")
        self.conv3 = ConvBNAct(width, cout, 1, act=None)
        self.down = ConvBNAct(cin, cout, 1, stride, act=None) if downsample else None
        self.stride, self.dilation = stride, dilation

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = self.conv3(self.conv2(self.conv1(x)))
        return torch.relu(y + idt)


class ResNet50Backbone(nn.Module):
    LAYERS = (3, 4, 6, 3)
    WIDTHS = (64, 128, 256, 512)

    def __init__(self, output_stride: int = 16, multi_grid: Tuple[int, ...] = (1, 2, 4)):
        super().__init__()
        self.stem = ConvBNAct(3, 64, 7, 2, act="relu")
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        if output_stride == 16:
            strides, dils = (1, 2, 2, 1), (1, 1, 1, 2)
        elif output_stride == 8:
            strides, dils = (1, 2, 1, 1), (1, 1, 2, 4)
        elif output_stride == 32:
            strides, dils = (1, 2, 2, 2), (1, 1, 1, 1)
        else:
            raise ValueError(output_stride)
        blocks: List[Bottleneck] = []
        cin = 64
        for li, (n, w) in enumerate(zip(self.LAYERS, self.WIDTHS)):
            for i in range(n):
                d = dils[li]
                if li == 3 and output_stride != 32 and multi_grid:
                    d = dils[li] * multi_grid[i % len(multi_grid)]
                blocks.append(Bottleneck(cin, w, strides[li] if i == 0 else 1, d, i == 0))
                cin = w * 4
        self.blocks = nn.ModuleList(blocks)
        self.out_channels = cin
        self.output_stride = output_stride

    def forward(self, x):
        x = self.maxpool(self.stem(x))
        for b in self.blocks:
            x = b(x)
        return x
