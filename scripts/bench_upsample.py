"""Microbench of the upsample+argmax kernel variants on the headline shape
(B=32, 33x33x21 bf16 logits -> 513x513 uint8 labels); checks every variant against
the row-block kernel and prints mean time per launch (HIP events). Two logit fields:
``noise`` (i.i.d. per source pixel: the argmax changes between most neighbouring source
pixels, as with the random-init benchmark model) and ``smooth`` (a 5x5 random field
upsampled to 33x33: a few large regions per frame, as a trained model's maps)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from semantic_segmentation_server_amd.ops import hip_ops as K  # noqa: E402


def main(B=32, h=33, H=513, C=21):
    ldk = (C + 7) // 8 * 8
    g = torch.Generator().manual_seed(0)
    noise = torch.randn(B, h, h, ldk, generator=g) * 2
    coarse = torch.randn(B, ldk, 5, 5, generator=g) * 4
    smooth = torch.nn.functional.interpolate(coarse, size=(h, h), mode="bilinear",
                                             align_corners=True).permute(0, 2, 3, 1)
    for field, lg in (("noise", noise), ("smooth", smooth)):
        print(f"-- {field}")
        run(lg.contiguous().to(torch.bfloat16).cuda(), B, h, H, C, ldk)
    return 0


def run(logits, B, h, H, C, ldk):
    outs = {}
    for name, v in K.UPSAMPLE_VARIANTS.items():
        out = torch.empty(B, H, H, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            K.upsample_argmax(logits, out, B=B, h=h, w=h, K=C, ldk=ldk, H=H, W=H, variant=v)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        st.record()
        for _ in range(n):
            K.upsample_argmax(logits, out, B=B, h=h, w=h, K=C, ldk=ldk, H=H, W=H, variant=v)
        en.record()
        en.synchronize()
        outs[name] = out
        agree = (out == outs["rows"]).float().mean().item() if "rows" in outs else 1.0
        print(f"{name:9s} {st.elapsed_time(en) / n * 1e3:8.1f} us  agree(rows)={agree:.6f}", flush=True)


if __name__ == "__main__":
    sys.exit(main())
