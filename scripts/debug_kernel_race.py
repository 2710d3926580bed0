"""Single-kernel concurrency check: three copies of ONE kernel (own buffers) launched on three
streams at once, many times; outputs compared with the sequential result. Kernels: depthwise
(VALU only), conv_gemm 1x1 (LDS-DMA GEMM), pw_conv, upsample_argmax."""
import os
import sys

import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
from semantic_segmentation_server_amd.ops import hip_ops as K  # noqa: E402

dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(0)
B, H, W, C, N = 2, 33, 33, 320, 256
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200


def mk(*shape, dtype=torch.bfloat16):
    return (torch.randn(*shape, generator=g) * 0.5).to(dtype).to(dev)


cases = {}
xs = [mk(B, H, W, C) for _ in range(3)]
w9 = mk(9, C, dtype=torch.float32)
b9 = mk(C, dtype=torch.float32)
outs = [torch.empty(B, H, W, C, dtype=torch.bfloat16, device=dev) for _ in range(3)]
cases["depthwise"] = (lambda i: K.depthwise3x3(xs[i], w9, b9, outs[i], B=B, IH=H, IW=W, C=C, OH=H, OW=W,
                                                 stride=1, dil=2, act="relu6"), outs)
wg = mk(N, 1, 1, C)
bg = mk(N, dtype=torch.float32)
og = [torch.empty(B, H, W, N, dtype=torch.bfloat16, device=dev) for _ in range(3)]
cases["conv_gemm1x1"] = (lambda i: K.conv_gemm(xs[i], wg, bg, og[i], B=B, IH=H, IW=W, Cin=C, OH=H, OW=W,
                                                Cout=N, k=1, act="relu"), og)
w3 = mk(N, 3, 3, C)
o3 = [torch.empty(B, H, W, N, dtype=torch.bfloat16, device=dev) for _ in range(3)]
cases["conv_gemm3x3d6"] = (lambda i: K.conv_gemm(xs[i], w3, bg, o3[i], B=B, IH=H, IW=W, Cin=C, OH=H, OW=W,
                                                  Cout=N, k=3, dil=6, act="relu"), o3)
wpk = K.pack_pw_weights(wg[:, 0, 0, :], bg)
op = [torch.empty(B * H * W, N, dtype=torch.bfloat16, device=dev) for _ in range(3)]
cases["pw_conv"] = (lambda i: K.pw_conv(xs[i], wpk, op[i], M=B * H * W, K=C, N=N, act="relu6", mt=2, nch=2), op)
ss = [torch.cuda.Stream() for _ in range(3)]
for name, (run, bufs) in cases.items():
    for i in range(3):
        run(i)
    torch.cuda.synchronize()
    ref = [b.clone() for b in bufs]
    bad = 0
    for r in range(reps):
        for i in range(3):
            bufs[i].fill_(0)
        torch.cuda.synchronize()
        for i in range(3):
            with torch.cuda.stream(ss[i]):
                run(i)
        torch.cuda.synchronize()
        bad += sum(int(not torch.equal(bufs[i], ref[i])) for i in range(3))
    print(f"{name}: {bad} / {3 * reps} concurrent runs differ", flush=True)
