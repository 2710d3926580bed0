"""hipBLASLt (torch.mm) time on the MobileNetV2 1x1 expand/project GEMM shapes at B=32,
to compare against the hand-written pw_conv / dw_proj kernels (layer_times)."""
import torch

shapes = [("b7-10 expand", 32 * 33 * 33, 64, 384), ("b11-13 expand", 32 * 33 * 33, 96, 576),
          ("b14-16 expand", 32 * 33 * 33, 160, 960), ("b14 project", 32 * 33 * 33, 960, 160),
          ("b4 expand 65^2", 32 * 65 * 65, 32, 192), ("aspp proj", 32 * 33 * 33, 1280, 256)]
for name, M, K, N in shapes:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16).t().contiguous()
    for layout, bb in (("NN", b), ("NT", b.t().contiguous().t())):
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(5):
            torch.mm(a, bb, out=out)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(50):
            torch.mm(a, bb, out=out)
        en.record()
        en.synchronize()
        us = st.elapsed_time(en) / 50 * 1e3
        gb = (M * K + K * N + M * N) * 2 / 1e9
        print(f"{name:16s} {layout} M={M} K={K} N={N}: {us:7.1f} us  {2*M*K*N/us/1e6:6.1f} TF/s  {gb/us*1e3:5.2f} TB/s", flush=True)
