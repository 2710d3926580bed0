"""Per-layer roofline of config 4 (DeepLabv3-ResNet50, 1025^2, int8, B frames) from a
rocprofv3 kernel trace: the int8 conv kernels of one step in plan order (stem, then per
bottleneck conv1, conv2, [down], conv3, then the ASPP 1x1 + three atrous branches, the
projection and the logits), each layer's MACs and minimal HBM bytes (int8 activations
in + out, int8 weights), achieved TOPS and the share of the MI355X dense int8 MFMA peak
(~5 POPS: twice the bf16 rate, MI355X_MICROARCH.md) and of the achievable HBM rate
(6.3 TB/s).

  python scripts/roofline_int8.py <run_kernel_trace.csv> [B] > profiles/r3_config4_roofline.txt"""
import csv
import sys

PEAK_TOPS, HBM = 5000.0, 6.3e12
path = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8


def layers(H=1025):
    out = []
    h = (H + 2 * 3 - 7) // 2 + 1                 # stem 7x7 s2
    out.append(("stem 7x7/2 3->64", h * h * 64 * 3 * 49, 3 * H * H + h * h * 64, 64 * 147))
    h = (h + 2 - 3) // 2 + 1                     # maxpool
    cin = 64
    cfg = [(3, 64, 1, [1, 1, 1]), (4, 128, 2, [1] * 4), (6, 256, 2, [1] * 6), (3, 512, 1, [2, 4, 8])]
    for li, (n, w, s, dils) in enumerate(cfg):
        for i in range(n):
            st = s if i == 0 else 1
            oh = (h - 1) // st + 1
            cout = 4 * w
            tag = f"L{li + 1}.{i}"
            out.append((f"{tag} conv1 1x1 {cin}->{w}", h * h * w * cin, h * h * (cin + w), cin * w))
            out.append((f"{tag} conv2 3x3/{st} d{dils[i]} {w}->{w}", oh * oh * w * w * 9, h * h * w + oh * oh * w, 9 * w * w))
            if i == 0:
                out.append((f"{tag} down 1x1/{st} {cin}->{cout}", oh * oh * cout * cin, h * h * cin + oh * oh * cout, cin * cout))
            out.append((f"{tag} conv3 1x1 {w}->{cout}", oh * oh * cout * w, oh * oh * (w + cout), w * cout))
            h, cin = oh, cout
    hw = h * h
    out.append((f"aspp 1x1 {cin}->256", hw * 256 * cin, hw * (cin + 256), cin * 256))
    for r in (6, 12, 18):
        out.append((f"aspp 3x3 d{r} {cin}->256 (all taps)", hw * 256 * cin * 9, hw * (cin + 256), 9 * cin * 256))
    out.append(("aspp proj 1024->256", hw * 256 * 1024, hw * (1024 + 256), 1024 * 256))
    out.append(("logits 256->19", hw * 19 * 256, hw * (256 + 19), 256 * 19))
    return out


rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "upsample_argmax" in r["Kernel_Name"]]
step = rows[ends[-2] + 1:ends[-1] + 1]
convs = [r for r in step if ("conv_i8" in r["Kernel_Name"] or "stem" in r["Kernel_Name"])]
L = layers()
print(f"# config 4, B = {B}: {len(convs)} conv kernels in the step, {len(L)} conv layers")
print(f"{'layer':44s} {'kernel':28s} {'us':>8s} {'GMAC':>8s} {'TOPS':>8s} {'%peak':>6s} {'MB':>8s} {'%HBM':>6s}")
tu = tm = 0.0
li = 0
for r in convs:
    if li >= len(L):
        break
    name, macs, act, wts = L[li]
    li += 1
    if "group" in r["Kernel_Name"] and name.startswith("aspp 1x1"):
        # the grouped ASPP launch: the 1x1 and the three atrous branches in one grid
        for _ in range(3):
            _, m2, a2, w2 = L[li]
            li += 1
            macs, wts = macs + m2, wts + w2
        name = "aspp 1x1 + 3x3 d6/12/18 (grouped, all taps)"
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("ssa::", "").split("(")[0]
    m = macs * B
    by = act * B + wts
    tops = 2 * m / (us * 1e-6) / 1e12
    print(f"{name:44s} {kn[-28:]:28s} {us:8.1f} {m / 1e9:8.2f} {tops:8.1f} {100 * tops / PEAK_TOPS:6.1f} "
          f"{by / 1e6:8.1f} {100 * by / (us * 1e-6) / HBM:6.1f}")
    tu += us
    tm += m
print(f"{'total convs':44s} {'':28s} {tu:8.1f} {tm / 1e9:8.2f} {2 * tm / (tu * 1e-6) / 1e12:8.1f} "
      f"{100 * 2 * tm / (tu * 1e-6) / 1e12 / PEAK_TOPS:6.1f}")
allk = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in step)
print(f"# whole step kernel time {allk:.1f} us (post-processing, pool, upsample included); the atrous "
      f"MACs count every tap (the kernel skips all-padding taps per tile)")
