"""Building blocks shared by the backbones.

The reference runs an opaque Edge-TPU tflite graph (``sem_seg_server.py:238,264``);
we define the network explicitly. Every conv is ``ConvBNAct`` so that BatchNorm can
be folded into the conv weights/bias for inference (``fold``), which is what the
HIP executor consumes.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


def make_divisible(v: float, divisor: int = 8, min_value: Optional[int] = None) -> int:
    """Channel rounding used by MobileNetV2 for depth multipliers."""
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


ACTS = (None, "relu", "relu6")


def apply_act(x: torch.Tensor, act: Optional[str]) -> torch.Tensor:
    if act is None:
        return x
    if act == "relu":
        return F.relu(x)
    if act == "relu6":
        return F.relu6(x)
    raise ValueError(act)


class ConvBNAct(nn.Module):
    """conv(k, stride, dilation, groups) -> BatchNorm -> activation.

    ``padding`` is ``dilation * (k // 2)`` (symmetric "same" for odd inputs, which
    is what TF SAME gives on the 513 -> 257 -> 129 -> 65 -> 33 pyramid).
    """

    def __init__(self, cin: int, cout: int, k: int = 1, stride: int = 1, dilation: int = 1,
                 groups: int = 1, act: Optional[str] = "relu6", bias_only: bool = False):
        super().__init__()
        assert act in ACTS
        self.cin, self.cout, self.k = cin, cout, k
        self.stride, self.dilation, self.groups, self.act = stride, dilation, groups, act
        self.conv = nn.Conv2d(cin, cout, k, stride, dilation * (k // 2), dilation, groups,
                              bias=bias_only)
        # bias_only: plain conv with bias and no BN (logits layer)
        self.bn = None if bias_only else nn.BatchNorm2d(cout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.conv(x)
        if self.bn is not None:
            y = self.bn(y)
        return apply_act(y, self.act)

    @torch.no_grad()
    def fold(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """Return (weight [cout, cin/groups, k, k], bias [cout]) in fp32 with BN folded."""
        w = self.conv.weight.detach().float()
        if self.bn is None:
            b = self.conv.bias.detach().float() if self.conv.bias is not None else torch.zeros(self.cout)
            return w.clone(), b.clone()
        bn = self.bn
        scale = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
        w = w * scale.view(-1, 1, 1, 1)
        b = bn.bias.float() - bn.running_mean.float() * scale
        if self.conv.bias is not None:
            b = b + self.conv.bias.float() * scale
        return w, b


def init_random(module: nn.Module, seed: int = 0) -> None:
    """Deterministic random init (north-star: random-init weights)."""
    g = torch.Generator().manual_seed(seed)
    for m in module.modules():
        if isinstance(m, nn.Conv2d):
            fan_in = m.in_channels // m.groups * m.kernel_size[0] * m.kernel_size[1]
            std = (2.0 / fan_in) ** 0.5
            with torch.no_grad():
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * std)
                if m.bias is not None:
                    m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)
        elif isinstance(m, nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.copy_(1.0 + 0.1 * torch.randn(m.weight.shape, generator=g))
                m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=g))
                m.running_mean.zero_()
                m.running_var.fill_(1.0)


@torch.no_grad()
def calibrate_bn(model: nn.Module, x: torch.Tensor) -> None:
    """Set BN running statistics from a synthetic batch.

    With random weights, unnormalised activations drift by orders of magnitude
    over ~60 layers; calibrating the running stats once (cumulative average in
    train mode) keeps every layer's output O(1), which keeps bf16 numerics and
    the argmax meaningful. Runs in fp32.
    """
    was_training = model.training
    saved = {}
    for m in model.modules():
        if isinstance(m, nn.BatchNorm2d):
            saved[m] = m.momentum
            m.momentum = None
            m.reset_running_stats()
    model.train()
    model(x)
    for m, mom in saved.items():
        m.momentum = mom
    model.train(was_training)
