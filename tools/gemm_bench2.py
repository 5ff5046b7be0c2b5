"""rk_linear / rk_gemm timing (HIP events) at the training shapes of BST (configs[3]: rows = 2048 x 64,
d_model 128) and DIN (att-MLP rows = 4096 x 50, widths 128 -> 64 -> 32)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd")
import rankops  # noqa: E402
from rankops import ops  # noqa: E402


def t(fn, it=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    rankops.load_library()
    for M, N, K in [(131072, 128, 128), (131072, 384, 128), (204800, 64, 128), (204800, 32, 64), (4096, 512, 128),
                    (4096, 256, 512)]:
        x = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda")
        y = torch.empty(M, N, device="cuda")
        us = t(lambda: ops.linear(x, w, y))
        print(f"linear M={M} N={N} K={K}: {us:.1f} us, {2 * M * N * K / us / 1e6:.1f} TFLOP/s, "
              f"{4 * (M * K + M * N) / us / 1e3:.0f} GB/s", flush=True)
    for TA, TB, M, N, R in [(0, 1, 131072, 128, 128), (1, 1, 128, 128, 131072), (0, 1, 204800, 128, 64),
                            (1, 1, 64, 128, 204800), (0, 1, 4096, 512, 256), (1, 1, 256, 512, 4096)]:
        A = torch.randn((R, M) if TA else (M, R), device="cuda")
        B = torch.randn((R, N) if TB else (N, R), device="cuda")
        C = torch.empty(M, N, device="cuda")
        us = t(lambda: ops.gemm(TA, TB, M, N, R, A, A.stride(0), B, B.stride(0), C))
        print(f"gemm TA={TA} TB={TB} M={M} N={N} R={R}: {us:.1f} us, {2 * M * N * R / us / 1e6:.1f} TFLOP/s",
              flush=True)


if __name__ == "__main__":
    main()
