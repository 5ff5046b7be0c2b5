"""rk_mlp_forward (streamed plans) at large batches with 16- vs 32-row workgroups
(RANKOPS_MLP_ROWS): average launch time over back-to-back launches, HIP events on the stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd"))
from rankops import ops  # noqa: E402
import rankops  # noqa: E402

rankops.load_library()
dev = torch.device("cuda")
g = torch.Generator().manual_seed(1)
for K0, widths in ((50, (512, 256, 128)), (114, (512, 256, 128)), (512, (256, 128))):
    mls, keep, k = [], [], K0
    for n in widths:
        w = ((torch.rand(n, k, generator=g) - 0.5) * (2.0 / k ** 0.5)).to(dev)
        b = (torch.rand(n, generator=g) - 0.5).to(dev)
        pk = ops.pack_mlp_weight(w)
        mls.append(ops.make_mlp_layer(w, pk, bias=b, act="relu"))
        keep += [w, b, pk]
        k = n
    hw = (torch.rand(widths[-1], generator=g) - 0.5).to(dev)
    hb = torch.tensor([0.05], device=dev)
    for M in (4096, 16384, 65536):
        x = (torch.rand(M, K0, generator=g) * 2 - 1).to(dev)
        logit = torch.empty(M, device=dev)
        ep = ops.make_epilogue(head_w=hw, head_b=hb, head_logit=logit)
        res = {}
        for rows in ("16", "32"):
            os.environ["RANKOPS_MLP_ROWS"] = rows
            for _ in range(5):
                ops.mlp_forward(x, mls, ep)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.mlp_forward(x, mls, ep)
            e1.record()
            torch.cuda.synchronize()
            res[rows] = e0.elapsed_time(e1) / 20 * 1e3
        print(f"K0 {K0:4d} {widths} M {M:6d}: 16 rows {res['16']:8.1f} us  32 rows {res['32']:8.1f} us  "
              f"({res['16'] / res['32']:.2f}x)", flush=True)
