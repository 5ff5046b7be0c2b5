"""Phase split of din_forward_kernel<32> at the bench's DIN configs[2] workload, from a timing
build of the library (make EXTRA=-DRK_DIN_PHASES OUT=<lib> BUILD=build_phases; point RANKOPS_LIB
at it).  Per workgroup: wall-clock (100 MHz) marks at entry, after staging, after phase A
(attention), after phase B (fcn tail); per wave: phase-A cycles.  Prints the distributions."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

batch = int(os.environ.get("BATCH", "4096"))
model, inp, fn, cfg, name = bench.workload("din", batch, 0)
launch = model.fused_kernel_launcher(inp["dense"], inp["category"], inp["sequence"], inp["target"])
us = 1e3 * bench.kernel_avg_ms(launch)
torch.cuda.synchronize()
n_launch = 5 + 50 + 1  # kernel_avg_ms warm-up + timed, and the launch below (RK_MLP_PHASES accumulates)
launch()
torch.cuda.synchronize()
from rankops import _lib  # noqa: E402
lib = _lib.load()
ts = (ctypes.c_ulonglong * (1024 * 8))()
wv = (ctypes.c_ulonglong * (1024 * 16))()
ml = (ctypes.c_ulonglong * (1024 * (4 * 8 + 4)))()
lib.rk_debug_din_phases.argtypes = [ctypes.c_void_p] * 3
assert lib.rk_debug_din_phases(ts, wv, ml) == 0
nwg = min(1024, (batch + 15) // 16)
t = np.array(ts, dtype=np.int64).reshape(1024, 8)[:nwg] * 10  # ns
w = np.array(wv, dtype=np.int64).reshape(1024, 16)[:nwg]
t0 = t[:, 0].min()
rel = (t - t0) / 1e3  # us from the first workgroup's entry
lens = inp["sequence"]["his_read_comment_7d_seq_length"].cpu().numpy()


def q(x):
    return f"min {np.min(x):7.2f}  med {np.median(x):7.2f}  max {np.max(x):7.2f}"


print(f"kernel avg {us:.2f} us (events), {nwg} workgroups")
print("entry        ", q(rel[:, 0]))
print("staging      ", q((t[:, 1] - t[:, 0]) / 1e3))
print("  image copied", q((t[:, 5] - t[:, 0]) / 1e3), "(tid 0, from entry)")
print("  counted     ", q((t[:, 6] - t[:, 0]) / 1e3), "(tid 0, from entry)")
print("assignment   ", q((t[:, 4] - t[:, 1]) / 1e3), "(wave 0)")
print("  A.1 (wave 0)", q((t[:, 7] - t[:, 4]) / 1e3), "(row + first keys loaded, from assignment)")
print("phase A      ", q((t[:, 2] - t[:, 1]) / 1e3))
print("phase B      ", q((t[:, 3] - t[:, 2]) / 1e3))
print("end          ", q(rel[:, 3]))
print("wave A cycles", q(w.reshape(-1) / 1e3), "(k cycles)")
print("wave A max/mean per WG", q(w.max(1) / np.maximum(w.mean(1), 1)))
print("lengths: mean", lens.mean(), "frac <= 32:", (lens <= 32).mean())
mlp = np.array(ml, dtype=np.float64).reshape(1024, 4 * 8 + 4)[:nwg] / 1e3
if mlp.any():
    print(f"phase B prologue {np.median(mlp[:, 32]):6.2f}k cycles (median over workgroups, wave 0)")
    for l in range(3):
        print(f"layer {l}: mfma issued {q(mlp[:, 4*l])} | epilogue {q(mlp[:, 4*l+1])} | prepare {q(mlp[:, 4*l+2])} | barrier {q(mlp[:, 4*l+3])}")
# workgroup imbalance: the number of 2-tile samples per workgroup against its phase-A and end times
# (contiguous 16-sample blocks only: RANKOPS_DIN_BALANCE=0)
if os.environ.get("RANKOPS_DIN_BALANCE", "1") != "0":
    sys.exit(0)
tiles = np.minimum((np.minimum(lens, 50) + 31) // 32, 2)[: nwg * 16].reshape(nwg, 16)
k2 = (tiles == 2).sum(1)
pa = (t[:, 2] - t[:, 1]) / 1e3
print("2-tile samples per WG:", q(k2), "| corr(k2, phase A) =", f"{np.corrcoef(k2, pa)[0, 1]:.3f}",
      "| corr(k2, end) =", f"{np.corrcoef(k2, rel[:, 3])[0, 1]:.3f}")
for kk in sorted(set(k2.tolist())):
    sel = k2 == kk
    print(f"  k2={kk:2d}: {sel.sum():3d} WGs, phase A med {np.median(pa[sel]):6.2f} us, end med {np.median(rel[sel, 3]):6.2f}")
