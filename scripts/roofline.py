"""Per-layer roofline of the headline step (DeepLabv3-MobileNetV2, 513^2, B frames) from a
rocprofv3 kernel trace: for every model layer the kernels that implement it, their time,
the layer's FLOPs and its minimal HBM traffic (layer input + output activations + weights,
bf16; a fused block's expanded tensor never leaves the CU, so it is not counted), the
achieved rates and their share of the MI355X dense bf16 MFMA peak (2.5 PFLOP/s) and of
the achievable HBM bandwidth (6.3 TB/s, MI355X_MICROARCH.md).

  python scripts/roofline.py <run_kernel_trace.csv> [--B 32] > profiles/<tag>_roofline.txt
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK_TFLOPS = 2500.0
HBM_TBS = 6.3


def layer_costs(B: int):
    """{layer: (MACs, activation bytes in+out, weight bytes)} for one B-frame step."""
    import torch
    from semantic_segmentation_server_amd.models.deeplab import build_model
    model = build_model("mnv2", 21, calibrate_hw=None).eval()
    acc = {}

    def key_of(name):
        p = name.split(".")
        if p[0] == "backbone":
            return "stem" if p[1] == "stem" else f"block{p[2]}"
        if p[0] == "aspp":
            return {"b0": "aspp.branches", "atrous": "aspp.branches", "pool": "aspp.pool",
                    "project": "aspp.head"}[p[1]]
        return "aspp.head"  # logits: fused into the head kernel

    hooks = []
    for name, m in model.named_modules():
        if isinstance(m, torch.nn.Conv2d):
            def hook(mod, inp, out, k=key_of(name), leaf=name):
                x = inp[0]
                kh, kw = mod.kernel_size
                taps = kh * kw
                if kh == 3 and mod.stride == (1, 1) and mod.dilation[0] > 1:
                    # atrous 'same' conv: count only in-image taps (padding taps multiply
                    # zeros; the kernels skip them)
                    H, W = out.shape[-2:]
                    d = mod.dilation[0]
                    cy = sum(sum(0 <= y + o < H for o in (-d, 0, d)) for y in range(H)) / H
                    cx = sum(sum(0 <= x + o < W for o in (-d, 0, d)) for x in range(W)) / W
                    taps = cy * cx
                macs = out.numel() * (mod.in_channels // mod.groups) * taps
                wbytes = mod.weight.numel() * 2
                a = acc.setdefault(k, {"macs": 0, "w": 0, "io": {}})
                a["macs"] += macs * B
                a["w"] += wbytes
                a["io"][leaf] = (x.numel() * B * 2, out.numel() * B * 2)
            hooks.append(m.register_forward_hook(hook))
    with torch.no_grad():
        model(torch.zeros(1, 3, 513, 513))
    for h in hooks:
        h.remove()
    out = {}
    for k, a in acc.items():
        ios = list(a["io"].values())
        # block-level traffic: first conv's input + last conv's output (intermediates fused)
        act = ios[0][0] + ios[-1][1] if k not in ("aspp.branches",) else ios[0][0] + sum(o for _, o in ios)
        out[k] = (a["macs"], act, a["w"])
    out["upsample+argmax"] = (B * 513 * 513 * 21 * 2, B * 33 * 33 * 24 * 2 + B * 513 * 513, 0)
    return out


def assign(rows):
    """Walk one step's kernels in launch order and attribute them to layers."""
    blocks = iter(range(1, 17))
    out = []
    i = 0
    while i < len(rows):
        n, us = rows[i]
        if n.startswith("__amd") or n.startswith("k_"):
            i += 1
            continue
        if n.startswith("stem_block0"):
            out.append(("stem+block0", [n], us))
        elif n.startswith("pw_conv") and i + 1 < len(rows) and rows[i + 1][0].startswith("dw_proj"):
            out.append((f"block{next(blocks)}", [n, rows[i + 1][0]], us + rows[i + 1][1]))
            i += 1
        elif n.startswith(("fused_ir", "conv_gemm_kernel", "dw3x3")):
            out.append((f"block{next(blocks)}", [n], us))
        elif n.startswith("conv_glds_group"):
            out.append(("aspp.branches", [n], us))
        elif n.startswith(("gap_partial", "aspp_pool")):
            if out and out[-1][0] == "aspp.pool":
                out[-1] = ("aspp.pool", out[-1][1] + [n], out[-1][2] + us)
            else:
                out.append(("aspp.pool", [n], us))
        elif n.startswith("aspp_head"):
            out.append(("aspp.head", [n], us))
        elif n.startswith("upsample"):
            out.append(("upsample+argmax", [n], us))
        i += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--B", type=int, default=32)
    a = ap.parse_args()
    sys.argv = [sys.argv[0], a.trace]
    import runpy
    import io
    import contextlib
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        lt = runpy.run_path(os.path.join(ROOT, "scripts", "layer_times.py"), run_name="lt")
    rows = lt["one_step"](a.trace)
    costs = layer_costs(a.B)
    # stem + block 0 fused: reads the uint8 640x480 camera frames, writes block 0's output
    cam = a.B * 480 * 640 * 3
    blk0_out = a.B * 257 * 257 * 16 * 2
    costs["stem+block0"] = (costs["stem"][0] + costs["block0"][0], cam + blk0_out,
                            costs["stem"][2] + costs["block0"][2])
    table = assign(rows)
    print(f"# per-layer roofline, DeepLabv3-MobileNetV2 513^2, B = {a.B}, from {os.path.basename(a.trace)}")
    print(f"# peaks: bf16 dense MFMA {PEAK_TFLOPS:.0f} TFLOP/s, HBM {HBM_TBS} TB/s achievable; "
          "min bytes = layer input + output activations + weights (bf16); atrous convs count "
          "in-image taps only")
    print(f"{'layer':16s} {'us':>7s} {'GFLOP':>7s} {'TFLOP/s':>8s} {'%MFMA':>6s} {'minMB':>7s} {'TB/s':>6s} "
          f"{'%HBM':>5s}  kernels")
    tus = tfl = 0.0
    for layer, ks, us in table:
        macs, act, w = costs.get(layer, (0, 0, 0))
        fl = 2 * macs / 1e9
        mb = (act + w) / 1e6
        tf = fl / us * 1e3 if us else 0.0  # GFLOP / us = PFLOP/s -> x1000 TFLOP/s
        tbs = mb / us if us else 0.0       # MB / us = TB/s
        tus += us
        tfl += fl
        print(f"{layer:16s} {us:7.1f} {fl:7.1f} {tf:8.1f} {100 * tf / PEAK_TFLOPS:5.1f}% {mb:7.1f} {tbs:6.2f} "
              f"{100 * tbs / HBM_TBS:4.0f}%  {' + '.join(k.split('<')[0] for k in ks)}")
    print(f"{'model total':16s} {tus:7.1f} {tfl:7.1f} {tfl / tus * 1e3:8.1f} {100 * tfl / tus * 1e3 / PEAK_TFLOPS:5.1f}%")


if __name__ == "__main__":
    main()
