"""Post-training int8 quantisation of DeepLabv3-ResNet50 (BASELINE config 4).

Scheme (symmetric, static):
  * weights: int8 per output channel, s_w[n] = max|W[n]| / 127 (BN folded first);
  * activations: int8 per tensor at every conv output, s_a = max|a| / 127 over
    a calibration batch of synthetic frames (post-ReLU tensors use [0, 127]);
  * every conv: exact int32 accumulation on the int8 MFMA, then
    v = acc * s_in * s_w[n] + bias (+ residual_int8 * s_res), ReLU, requantise.
  * ASPP branches share one concat scale; the image-pooling branch stays fp32
    (it enters the projection as a per-image bias); the logits layer outputs bf16.

``fake_quant_forward`` replays exactly this arithmetic in fp32 torch and is the
numerics reference for the HIP int8 path (tests/test_hip_kernels.py).
The reference server has no quantisation code of its own: its Edge-TPU model is
a uint8 tflite compiled offline (sem_seg_server.py:238).
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from .deeplab import DeepLabV3
from .layers import ConvBNAct
from .resnet import ResNet50Backbone


def _qw(layer: ConvBNAct):
    w, b = layer.fold()
    amax = w.abs().amax(dim=(1, 2, 3)).clamp(min=1e-8)
    sw = amax / 127.0
    wq = torch.clamp(torch.round(w / sw.view(-1, 1, 1, 1)), -127, 127)
    return wq, sw, b


def q(x: torch.Tensor, s: float) -> torch.Tensor:
    """Quantise-dequantise with a per-tensor scale (round half to even like rintf)."""
    return torch.clamp(torch.round(x / s), -127, 127) * s


@torch.no_grad()
def calibrate(model: DeepLabV3, x: torch.Tensor) -> Dict[str, float]:
    """Activation scales (amax / 127) at every quantisation point, fp32 forward."""
    bb = model.backbone
    assert isinstance(bb, ResNet50Backbone), "int8 path is for DeepLabv3-ResNet50"
    amax: Dict[str, float] = {}

    def upd(name, t):
        amax[name] = max(amax.get(name, 0.0), float(t.abs().max()))

    h = bb.stem(x)
    upd("stem", h)
    h = bb.maxpool(h)
    for i, blk in enumerate(bb.blocks):
        idt = h if blk.down is None else blk.down(h)
        if blk.down is not None:
            upd(f"b{i}.down", idt)
        t1 = blk.conv1(h)
        upd(f"b{i}.c1", t1)
        t2 = blk.conv2(t1)
        upd(f"b{i}.c2", t2)
        h = torch.relu(blk.conv3(t2) + idt)
        upd(f"b{i}.out", h)
    a = model.aspp
    outs = [a.b0(h)] + [br(h) for br in a.atrous]
    for o in outs:
        upd("aspp.cat", o)
    p = a.pool(F.adaptive_avg_pool2d(h, 1))
    proj = a.project(torch.cat(outs + [p.expand(-1, -1, h.shape[2], h.shape[3])], 1))
    upd("aspp.proj", proj)
    return {k: max(v, 1e-6) / 127.0 for k, v in amax.items()}


@torch.no_grad()
def fake_quant_forward(model: DeepLabV3, scales: Dict[str, float], x: torch.Tensor,
                       stem_bf16: bool = False) -> torch.Tensor:
    """fp32 replay of the int8 pipeline -> logits (N, K, h, w). ``stem_bf16``: the stem as
    the MFMA stem kernels compute it (normalised pixels and folded weights rounded to bf16,
    fp32 accumulation, int8 out) instead of the fp32 per-lane stem: the int8 network
    amplifies a stem code that differs by one step into multi-step differences a few
    blocks later, so the replay must round where the plan's stem rounds."""
    bb = model.backbone

    def conv(layer: ConvBNAct, inp, s_out=None, res=None, act=None, quant_w=True):
        if quant_w:
            wq, sw, b = _qw(layer)
            wf = wq * sw.view(-1, 1, 1, 1)
        else:  # the fused stem: fp32 (or bf16-rounded) weights on fp32 (bf16) pixels
            wf, b = layer.fold()
            if stem_bf16:
                wf = wf.to(torch.bfloat16).float()
                inp = inp.to(torch.bfloat16).float()
        y = F.conv2d(inp, wf, b, layer.stride,
                     layer.dilation * (layer.k // 2), layer.dilation)
        if res is not None:
            y = y + res
        a = layer.act if act is None else act
        if a == "relu":
            y = torch.relu(y)
        return q(y, s_out) if s_out is not None else y

    h = conv(bb.stem, x, scales["stem"], quant_w=False)
    h = F.max_pool2d(h, 3, 2, 1)
    for i, blk in enumerate(bb.blocks):
        idt = h if blk.down is None else conv(blk.down, h, scales[f"b{i}.down"])
        t1 = conv(blk.conv1, h, scales[f"b{i}.c1"])
        t2 = conv(blk.conv2, t1, scales[f"b{i}.c2"])
        h = conv(blk.conv3, t2, scales[f"b{i}.out"], res=idt, act="relu")
    a = model.aspp
    outs = [conv(a.b0, h, scales["aspp.cat"])] + [conv(br, h, scales["aspp.cat"]) for br in a.atrous]
    pooled = a.pool(F.adaptive_avg_pool2d(h, 1))  # fp32 branch
    pw, pb = a.project.fold()
    ncat = len(outs) * a.cout
    wq_full, sw_full, _ = _qw(a.project)
    wq = wq_full[:, :ncat] * sw_full.view(-1, 1, 1, 1)
    img_bias = F.conv2d(pooled, pw[:, ncat:]).flatten(1)  # fp32 pool contribution
    proj = F.conv2d(torch.cat(outs, 1), wq, pb) + img_bias[:, :, None, None]
    proj = q(torch.relu(proj), scales["aspp.proj"])
    lq, ls, lb = _qw(model.logits)
    return F.conv2d(proj, lq * ls.view(-1, 1, 1, 1), lb)


@torch.no_grad()
def int8_conv_codes(layer: ConvBNAct, x_codes: torch.Tensor, s_in: float, s_out: float,
                    res_codes: torch.Tensor = None, s_res: float = 0.0, act: str = None,
                    chunk_k: int = 576) -> torch.Tensor:
    """One int8 conv of the plan in exact arithmetic, from the plan's OWN input codes
    (teacher forcing): integer accumulators exactly (fp32 convs over input-channel chunks
    whose partial sums stay below 2^24, summed in float64), then v = acc * s_in * s_w +
    bias (+ res * s_res), ReLU, round-half-even requantisation. x_codes / res_codes: NCHW
    integer-valued tensors; returns NCHW int32 codes. A kernel matches this up to rounding
    ties of its fp32 epilogue (a code off by one, rarely); the network itself amplifies such
    a flip into multi-step differences a few blocks later, so per-layer teacher-forced
    comparison is how a plan's kernels are checked at full depth."""
    wq, sw, b = _qw(layer)
    kk = layer.k * layer.k
    step = max(1, chunk_k // kk)  # input channels per chunk: step * k^2 * 127^2 < 2^24
    acc = None
    pad, dil = layer.dilation * (layer.k // 2), layer.dilation
    xf = x_codes.float()
    for c0 in range(0, xf.shape[1], step):
        part = F.conv2d(xf[:, c0:c0 + step], wq[:, c0:c0 + step].to(xf.device), None, layer.stride,
                        pad, dil).double()
        acc = part if acc is None else acc + part
    v = acc * (s_in * sw.double().to(acc.device)).view(1, -1, 1, 1) + b.double().to(acc.device).view(1, -1, 1, 1)
    if res_codes is not None:
        v = v + res_codes.double() * s_res
    a = layer.act if act is None else act
    if a == "relu":
        v = torch.relu(v)
    return torch.clamp(torch.round(v / s_out), -127, 127).to(torch.int32)


def pack_int8(layer: ConvBNAct, in_scale: float, device, wslice=None):
    """-> (w_int8 [Cout, kh, kw, Cin], combined scale [Cout] = s_in * s_w, bias [Cout])."""
    wq, sw, b = _qw(layer)
    if wslice is not None:
        wq = wq[:, wslice]
    w8 = wq.permute(0, 2, 3, 1).contiguous().to(torch.int8).to(device)
    return w8, (sw * in_scale).float().to(device), b.float().to(device)
