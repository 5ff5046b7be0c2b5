"""DCN eval forward (rk_dcn_forward, one launch) at large batches with 16- vs 32-row workgroups
(RANKOPS_MLP_ROWS): average step time over back-to-back forwards, CUDA events."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

for batch in (4096, 16384, 65536):
    res = {}
    for rows in ("16", "32"):
        os.environ["RANKOPS_MLP_ROWS"] = rows  # before the workload: no launch cache crosses settings
        model, inp, fn, cfg, name = bench.workload("dcn", batch, 0)
        with torch.no_grad():
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
        res[rows] = e0.elapsed_time(e1) / 20 * 1e3
    print(f"dcn batch {batch:6d}: 16 rows {res['16']:8.1f} us  32 rows {res['32']:8.1f} us  ({res['16'] / res['32']:.2f}x)",
          flush=True)
