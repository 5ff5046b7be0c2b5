"""gemm_rows at the BST training shape (M = 2048 x 64 rows, N = K = 128): the bias+ReLU linear
(EPI FAST) and the accumulating dX gemm (ACC FAST), 20 launches each, for counter passes
(tools/sq_pass.sh) and HIP-event timing."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd")
import rankops  # noqa: E402
from rankops import ops  # noqa: E402

import os  # noqa: E402

rankops.load_library()
M, N, K = int(os.environ.get("M", "131072")), 128, 128
x = torch.randn(M, K, device="cuda")
w = torch.randn(N, K, device="cuda")
b = torch.randn(N, device="cuda")
y = torch.empty(M, N, device="cuda")
ep = ops.make_epilogue(bias=b, act="relu")
dy = torch.randn(M, N, device="cuda")
dx = torch.zeros(M, K, device="cuda")


def lin():
    ops.linear(x, w, y, epilogue=ep)


def acc():
    ops.gemm(0, 0, M, K, N, dy, dy.stride(0), w, w.stride(0), dx, accumulate=True)


for name, fn in (("linear_bias_relu", lin), ("gemm_acc", acc)):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    print(f"{name}: {us:.1f} us  {2 * M * N * K / us / 1e6:.1f} TFLOP/s", flush=True)
