"""hipBLASLt (torch.matmul, bf16) on the model's plain-GEMM shapes, as a yardstick
for the hand-written kernels: M = 32 x 33 x 33 pixels."""
import torch


def bench(M, K, N, reps=20):
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        c = a @ b
    en.record()
    torch.cuda.synchronize()
    t = st.elapsed_time(en) / reps * 1e3
    print(f"M={M} K={K} N={N}: {t:7.1f} us  {2 * M * K * N / t / 1e6:6.0f} TF", flush=True)


M = 32 * 33 * 33
for K, N in ((1024, 256), (320, 256), (2880, 256), (160, 960), (960, 160), (960, 320), (96, 576), (576, 96)):
    bench(M, K, N)

# the projection as the model calls it: out= into a static buffer, weight as a transposed view
a = torch.randn(M, 1024, device="cuda", dtype=torch.bfloat16)
w = torch.randn(256, 1024, device="cuda", dtype=torch.bfloat16)
out = torch.empty(M, 256, device="cuda", dtype=torch.bfloat16)
for name, fn in (("view.t out=", lambda: torch.mm(a, w.t(), out=out)),
                 ("contig out=", lambda wt=w.t().contiguous(): torch.mm(a, wt, out=out)),
                 ("contig", lambda wt=w.t().contiguous(): torch.mm(a, wt))):
    for _ in range(3):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(20):
        fn()
    en.record()
    torch.cuda.synchronize()
    print(f"{name}: {st.elapsed_time(en) / 20 * 1e3:7.1f} us", flush=True)
