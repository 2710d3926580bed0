"""int8 DeepLabv3-ResNet50 on the gfx950 int8 MFMA kernels (BASELINE config 4).

Same interface as ``HipDeepLab`` (``segment`` / ``logits``). The plan:

  fused letterbox+stem conv (fp32 math, int8 out) -> int8 max pool
  -> 16 bottlenecks: conv1 1x1, conv2 3x3 (strided / dilated), [down 1x1],
     conv3 1x1 with the int8 identity fused as a dequantised residual, ReLU,
     requantised int8 out
  -> ASPP: 1x1 + three atrous 3x3 branches written into one int8 concat buffer
     (shared scale); image pooling in fp32 folded into the projection's per-image
     bias; projection int8 -> logits conv with bf16 output
  -> fused bilinear upsample + argmax.

Scales come from ``models.quant.calibrate`` on synthetic frames.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from ..ops import hip_ops as K
from ..ops.hip_ops import conv_out_hw
from .deeplab import DeepLabV3, synthetic_normalized
from .quant import calibrate, pack_int8


_I8_VARIANTS = (1, 2, 3, 4, 7, 8, 18, 19, 20)  # register-fed, LDS-DMA 128x128 / 128x256 / 256x128 /
# 160x128 / 96x128, and 18-20: 128x128 / 128x256 / 256x128 with 64-byte K rows per stage
# (12 / 13, the n-tile-major orders, timed within noise of 7 / 2 or slower: not offered)
# + 5 / 6: streaming 1x1 (weights resident per channel block, prefetched pixel tiles; 6 with
# a narrower channel block) where it fits


def I8(*args, **kw):
    """One int8 conv step as an autotuned Choice over the conv_i8 kernel variants."""
    from .hip_model import Choice
    I8.n = getattr(I8, "n", 0) + 1
    variants = list(_I8_VARIANTS)
    if K.conv_i8_1x1_ok(int8_out=kw.get("out_scale") is not None, **kw):
        variants += [5, 6, 10, 11]
    c = Choice(f"i8conv{I8.n}", [(f"v{v}", [lambda *_, v=v: K.conv_i8(*args, variant=v, **kw)])
                                 for v in variants])
    c.desc = (f"M={kw['B'] * kw['OH'] * kw['OW']} Cin={kw['Cin']} Cout={kw['Cout']} "
              f"k={kw.get('k', 1)} s={kw.get('stride', 1)} d={kw.get('dil', 1)}")
    return c


class HipDeepLabInt8:
    def __init__(self, model: DeepLabV3, device: torch.device, cfg=None,
                 scales: Optional[Dict[str, float]] = None, calib_hw: int = 257):
        self.device = device
        self.model = model
        self.H = self.W = int(cfg.input_size) if cfg is not None else 1025
        self.num_classes = model.num_classes
        self.ldk = (self.num_classes + 7) // 8 * 8
        if scales is None:
            x = synthetic_normalized(4, calib_hw, calib_hw, torch.Generator().manual_seed(11))
            m32 = model.float()
            if device.type == "cuda":
                import copy
                m32 = copy.deepcopy(model).float().to(device)
                x = x.to(device)
            scales = calibrate(m32, x)
        self.scales = scales
        S = scales
        dev = device
        bb = model.backbone
        sw, sb = bb.stem.fold()
        self.stem_w = sw.permute(2, 3, 1, 0).reshape(-1, sw.shape[0]).contiguous().to(dev, torch.float32)
        self.stem_b = sb.to(dev, torch.float32)
        self.stem_meta = (bb.stem.k, bb.stem.stride, bb.stem.cout)
        self.blocks = []
        s_in = S["stem"]  # max pool keeps the scale
        for i, blk in enumerate(bb.blocks):
            d = dict(blk=blk, s_in=s_in)
            d["c1"] = pack_int8(blk.conv1, s_in, dev)
            d["c2"] = pack_int8(blk.conv2, S[f"b{i}.c1"], dev)
            d["c3"] = pack_int8(blk.conv3, S[f"b{i}.c2"], dev)
            d["down"] = pack_int8(blk.down, s_in, dev) if blk.down is not None else None
            d["s_res"] = S[f"b{i}.down"] if blk.down is not None else s_in
            self.blocks.append(d)
            s_in = S[f"b{i}.out"]
        self.s_feat = s_in
        a = model.aspp
        self.A = a.cout
        self.aspp_b0 = pack_int8(a.b0, s_in, dev)
        self.aspp_atrous = [(pack_int8(br, s_in, dev), br.dilation) for br in a.atrous]
        self.cat_c = (1 + len(a.atrous)) * a.cout
        self.proj = pack_int8(a.project, S["aspp.cat"], dev, wslice=slice(0, self.cat_c))
        pw, _ = a.project.fold()
        self.proj_pool_w = pw[:, self.cat_c:, 0, 0].contiguous().to(dev, torch.float32)
        qw, qb = a.pool.fold()
        self.pool_w = qw[:, :, 0, 0].contiguous().to(dev, torch.float32)
        self.pool_b = qb.to(dev, torch.float32)
        self.logits_p = pack_int8(model.logits, S["aspp.proj"], dev)
        self._plans: Dict[tuple, Tuple[List[Callable], Dict[str, torch.Tensor]]] = {}
        self._labels_out: Optional[torch.Tensor] = None  # segment(out=): caller's label maps
        self.kind = "resnet50_int8"  # tune-file key prefix
        self.pick_sync = None  # set by the DP pipeline: rank 0's picks on every rank
        self.choices: Dict[str, str] = {}

    def _plan(self, B: int, Hc: int, Wc: int, part: int = 0):
        """``part`` > 0: an independent copy of the plan (own buffers, part 0's picks) for
        the engine's slot-parallel execution (hip_model.HipDeepLab._plan)."""
        key = (B, Hc, Wc) if part == 0 else (B, Hc, Wc, part)
        if key in self._plans:
            return self._plans[key]
        dev, S = self.device, self.scales
        bufs: Dict[str, torch.Tensor] = {}
        ops: List[Callable] = []
        I8.n = 0  # conv choices named i8conv1.. by position: stable keys for the tune file

        def buf(name, *shape, dtype=torch.int8):
            t = torch.zeros(shape, dtype=dtype, device=dev)  # plan copies start identical
            bufs[name] = t
            return t

        H, W = self.H, self.W
        k, st, c = self.stem_meta
        OH, OW = conv_out_hw(H, W, k, st, 1)
        x = buf("stem", B, OH, OW, c)
        from .hip_model import Choice
        stem_variants = [("fp32", [lambda frames, lx, ly, x=x, OH=OH, OW=OW, c=c: K.stem_conv(
            frames, lx, ly, self.stem_w, self.stem_b, x, H=H, W=W, OH=OH, OW=OW, Cout=c, k=k,
            stride=st, act="relu", out_scale=S["stem"])])]
        if (c, k) in ((64, 7), (32, 3)):
            # the dense stem on bf16 MFMA (int8 out): one LDS-gathered input tile per workgroup
            wpk = K.pack_stem_mfma(self.stem_w, k, c)
            bufs["stem_wpk"] = wpk
            for tile in ((8, 16), (16, 16), (4, 32)):
                stem_variants.append((f"mfma{tile[0]}x{tile[1]}", [
                    lambda frames, lx, ly, x=x, OH=OH, OW=OW, c=c, tile=tile, wpk=wpk: K.stem_mfma(
                        frames, lx, ly, wpk, self.stem_b, x, H=H, W=W, OH=OH, OW=OW, Cout=c, k=k,
                        stride=st, act="relu", out_scale=S["stem"], tile=tile)]))
            if (c, k) == (64, 7):  # one wave per 16 output channels (26 weight VGPRs, not 104)
                # (a letterbox pre-pass with dense tiles measured slower: 148.7 vs 127.9 us,
                # profiles/r8k_stem_prepass_negative.txt)
                for tile in ((16, 16), (16, 32), (32, 32)):
                    stem_variants.append((f"mfmaw{tile[0]}x{tile[1]}", [
                        lambda frames, lx, ly, x=x, OH=OH, OW=OW, c=c, tile=tile, wpk=wpk: K.stem_mfma(
                            frames, lx, ly, wpk, self.stem_b, x, H=H, W=W, OH=OH, OW=OW, Cout=c, k=k,
                            stride=st, act="relu", out_scale=S["stem"], tile=tile, per_wave=True)]))
        ops.append(Choice("stem", stem_variants))
        PH, PW = conv_out_hw(OH, OW, 3, 2, 1)
        y = buf("pool0", B, PH, PW, c)
        ops.append(lambda *_, x=x, y=y, OH=OH, OW=OW, PH=PH, PW=PW, c=c: K.maxpool3x3s2_i8(
            x, y, B=B, IH=OH, IW=OW, C=c, OH=PH, OW=PW))
        x, h, w = y, PH, PW
        for i, d in enumerate(self.blocks):
            x, h, w, c = self._block(ops, buf, i, d, x, B, h, w, c)
        # ASPP
        A = self.A
        cat = buf("aspp_cat", B, h, w, self.cat_c)
        s_cat = S["aspp.cat"]
        ops.append(self._aspp_branches(bufs, x, cat, B, h, w, c))
        gap = buf("gap", B, c, dtype=torch.float32)
        gws = buf("gap_ws", B * 16 * c, dtype=torch.float32)
        pooled = buf("pooled", B, A, dtype=torch.float32)
        img_bias = buf("img_bias", B, A, dtype=torch.float32)
        ops.append(lambda *_, x=x, h=h, w=w, c=c: K.global_avgpool_i8(
            x, gap, gws, B=B, HW=h * w, C=c, scale=self.s_feat))
        ops.append(lambda *_, c=c: K.matvec(gap, self.pool_w, self.pool_b, pooled, B=B, N=A, K=c,
                                            act="relu"))
        ops.append(lambda *_: K.matvec(pooled, self.proj_pool_w, None, img_bias, B=B, N=A, K=A))
        proj = buf("aspp_proj", B, h, w, A)
        pw8, psc, pb = self.proj
        ops.append(I8(
            cat, pw8, psc, pb, proj, B=B, IH=h, IW=w, Cin=self.cat_c, OH=h, OW=w, Cout=A,
            act="relu", img_bias=img_bias, out_scale=S["aspp.proj"]))
        logits = buf("logits", B, h, w, self.ldk, dtype=torch.bfloat16)
        lw8, lsc, lb = self.logits_p
        ops.append(I8(
            proj, lw8, lsc, lb, logits, B=B, IH=h, IW=w, Cin=A, OH=h, OW=w,
            Cout=self.num_classes, ldo=self.ldk, act=None))
        labels = buf("labels", B, H, W, dtype=torch.uint8)
        ops.append(lambda *_, h=h, w=w: K.upsample_argmax(
            logits, self._labels_out if self._labels_out is not None else labels, B=B, h=h, w=w,
            K=self.num_classes, ldk=self.ldk, H=H, W=W, variant=K.UPSAMPLE_VARIANTS["lane"]))
        self._plans[key] = (ops, bufs)
        if part == 0:
            self._autotune(ops, B, Hc, Wc)
        else:
            from .hip_model import _copy_picks
            _copy_picks(self._plan(B, Hc, Wc)[0], ops)
            dev = self.device
            args = (torch.zeros((B, Hc, Wc, 3), dtype=torch.uint8, device=dev),
                    torch.zeros(self.W, dtype=torch.int32, device=dev),
                    torch.zeros(self.H, dtype=torch.int32, device=dev))
            for op in ops:  # first launches outside any capture
                op(*args)
            torch.cuda.synchronize(dev)
        return self._plans[key]

    def _aspp_branches(self, bufs, x, cat, B, h, w, c):
        """The ASPP 1x1 + atrous branches into the int8 concat buffer, as a Choice between
        four separate LDS-DMA launches (160x128 tiles, raster rows) and ONE grouped launch per
        tile shape: the atrous rows permuted into tap-uniform tiles (``tap_group_perm``: at
        65 x 65 the rate-6/12/18 tiles skip every padding tap, 23 / 43 / 60 % of the raster
        work) and every branch's tiles in one heaviest-first order, so the light tiles fill
        the tail instead of each branch's grid idling on its own."""
        from .hip_model import Choice
        A, S = self.A, self.scales
        s_cat = S["aspp.cat"]
        w8, sc, bi = self.aspp_b0
        convs = [dict(x=x, w=w8, scale=sc, bias=bi, out=cat, B=B, IH=h, IW=w, Cin=c, OH=h, OW=w,
                      Cout=A, ldo=self.cat_c, co_off=0, act="relu", out_scale=s_cat)]
        for j, ((aw, asc, ab), rate) in enumerate(self.aspp_atrous):
            convs.append(dict(x=x, w=aw, scale=asc, bias=ab, out=cat, B=B, IH=h, IW=w, Cin=c, OH=h,
                              OW=w, Cout=A, k=3, dil=rate, ldo=self.cat_c, co_off=(j + 1) * A,
                              act="relu", out_scale=s_cat))

        def sep(cv, v):
            kw = {k: x for k, x in cv.items() if k not in ("x", "w", "scale", "bias", "out")}
            return lambda *_: K.conv_i8(cv["x"], cv["w"], cv["scale"], cv["bias"], cv["out"], variant=v, **kw)

        # separate launches (raster 160x128 tiles) or one grouped launch. Measured (r7d-r7g,
        # B = 8, 65 x 65): sep 481-487 us, grouped 476-551 us over the tile shapes and orders
        # (global LPT, branch-affine XCD sets per branch / per channel tile), n-tile-major
        # separate 524 us: the tap-uniform tiles cut the K steps but not the time, so the
        # grouped form stays an autotune candidate, not the default
        variants = [("sep", [sep(cv, 7) for cv in convs])]
        for v in (7,):
            BM = K.I8_TILE[v][0]
            gc = []
            for j, cv in enumerate(convs):
                cv = dict(cv)
                if cv.get("k", 1) > 1:
                    cv["perm"] = K.tap_group_perm(B, h, w, 3, cv["dil"], BM, device=self.device)
                    bufs[f"aspp_perm{j}_v{v}"] = cv["perm"]
                gc.append(cv)
            # branch-affine XCD sets, per branch / per branch channel tile
            for xcds, by_n, tag in ((8, False, "x"),):
                order = K.grouped_tile_order_i8(gc, v, device=self.device, xcds=xcds, by_n=by_n)
                bufs[f"aspp_order_v{v}{tag}"] = order
                variants.append((f"g{v}{tag}", [lambda *_, gc=gc, order=order, v=v: K.conv_i8_grouped(gc, order, v)]))
        ch = Choice("aspp_i8", variants)
        ch.desc = f"M={B * h * w} Cin={c} Cout={A} x {len(convs)} branches"
        return ch

    def _tune_inputs(self, B: int, Hc: int, Wc: int):
        from .hip_model import HipDeepLab
        return HipDeepLab._tune_inputs(self, B, Hc, Wc)

    def _autotune(self, ops, B, Hc, Wc) -> None:
        """The bf16 model's plan tuning (hip_model.HipDeepLab._autotune): picks from the
        committed tune file (key ``resnet50_int8:B=..:cam=..:in=..``) when it has this
        shape, else timed on synthetic frames through the real letterbox LUTs -- on rank 0
        only under the DP pipeline's ``pick_sync``, so every rank runs the same kernels (the
        int8 variants differ by up to one requantisation step) and no rank tunes cold."""
        from .hip_model import HipDeepLab
        HipDeepLab._autotune(self, ops, B, Hc, Wc)

    def _block(self, ops, buf, i, d, x, B, h, w, c):
        S = self.scales
        m = d["blk"]
        width, cout = m.conv1.cout, m.conv3.cout
        OH, OW = conv_out_hw(h, w, 3, m.stride, m.dilation)
        w1, s1, b1 = d["c1"]
        t1 = buf(f"r{i}_c1", B, h, w, width)
        ops.append(I8(
            x, w1, s1, b1, t1, B=B, IH=h, IW=w, Cin=c, OH=h, OW=w, Cout=width, act="relu",
            out_scale=S[f"b{i}.c1"]))
        w2, s2, b2 = d["c2"]
        t2 = buf(f"r{i}_c2", B, OH, OW, width)
        ops.append(I8(
            t1, w2, s2, b2, t2, B=B, IH=h, IW=w, Cin=width, OH=OH, OW=OW, Cout=width, k=3,
            stride=m.stride, dil=m.dilation, act="relu", out_scale=S[f"b{i}.c2"]))
        if d["down"] is not None:
            wd, sd, bd = d["down"]
            idt = buf(f"r{i}_down", B, OH, OW, cout)
            ops.append(I8(
                x, wd, sd, bd, idt, B=B, IH=h, IW=w, Cin=c, OH=OH, OW=OW, Cout=cout,
                stride=m.stride, act=None, out_scale=S[f"b{i}.down"]))
        else:
            idt = x
        w3, s3, b3 = d["c3"]
        out = buf(f"r{i}_out", B, OH, OW, cout)
        ops.append(I8(
            t2, w3, s3, b3, out, B=B, IH=OH, IW=OW, Cin=width, OH=OH, OW=OW, Cout=cout,
            act="relu", res=idt, res_scale=d["s_res"], out_scale=S[f"b{i}.out"]))
        return out, OH, OW, cout

    def segment(self, frames, lut_x, lut_y, out: Optional[torch.Tensor] = None, part: int = 0):
        B, Hc, Wc, _ = frames.shape
        ops, bufs = self._plan(B, Hc, Wc, part)
        if out is not None and (out.shape != bufs["labels"].shape or out.dtype != torch.uint8
                                or not out.is_contiguous()):
            raise ValueError("segment: out must match the (B, H, W) uint8 label buffer")
        frames = frames.contiguous()
        self._labels_out = out
        try:
            for op in ops:
                op(frames, lut_x, lut_y)
        finally:
            self._labels_out = None
        return bufs["labels"] if out is None else out

    def logits(self, frames, lut_x, lut_y):
        self.segment(frames, lut_x, lut_y)
        B, Hc, Wc, _ = frames.shape
        return self._plans[(B, Hc, Wc)][1]["logits"][..., : self.num_classes]
