"""DCN eval forward (rk_dcn_forward, one launch) with 16- vs 32-row workgroups (RANKOPS_DCN_ROW_TILES
= 1 / 2): device time per forward from 20 forwards captured in one hipGraph (bench.graph_kernel_avg_ms),
and the outputs of the two forms compared bit for bit."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    torch.cuda.set_device(0)
    import rankops
    rankops.load_library()
    import helpers as H
    for batch in (4096, 8192, 16384, 65536):
        model, inp, fn, cfg, name = bench.workload("dcn", batch, 0)
        res, outs = {}, {}
        for rt in ("1", "2"):
            os.environ["RANKOPS_DCN_ROW_TILES"] = rt
            model.__dict__.pop("_eager", None)
            with torch.no_grad():
                outs[rt] = tuple(o.clone() for o in H.as_tuple(fn()))
            res[rt] = bench.graph_kernel_avg_ms(fn) * 1e3
        same = all(torch.equal(a, b) for a, b in zip(outs["1"], outs["2"]))
        print(f"dcn batch {batch:6d}: 16 rows {res['1']:8.2f} us  32 rows {res['2']:8.2f} us  "
              f"({res['1'] / res['2']:.3f}x)  bit-identical {same}", flush=True)
        del model, inp
    os.environ.pop("RANKOPS_DCN_ROW_TILES", None)


if __name__ == "__main__":
    main()
