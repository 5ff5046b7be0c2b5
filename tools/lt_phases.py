"""Phase split of the 2D-tiled layer kernel (linear_tiled_kernel: DeepFM's fused front end
rk_fm_linear_packed, or rk_linear_tiled with FUSED_FRONT off) at the bench's batch, from a timing
build of the library (make EXTRA="-DRK_DIN_PHASES -DRK_MLP_PHASES" OUT=../rankops/librankops_phases.so
BUILD=build_phases; point RANKOPS_LIB at it).  Per workgroup, wave 0, cycles from kernel entry to:
prologue (row pointers), block 0 staged, each K-block's MFMAs issued / barrier passed, epilogue,
end; per wave: last block's MFMAs issued and epilogue stored."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

batch = int(os.environ.get("BATCH", "4096"))
model, inp, fn, cfg, _ = bench.workload("deepfm", batch, 0)
if os.environ.get("UNFUSED"):
    from rankops import deepfm as deepfm_mod
    deepfm_mod.FUSED_FRONT = False
g, _ = bench.graph_of(fn)
us = 1e3 * bench.kernel_avg_ms(g.replay)
g.replay()
torch.cuda.synchronize()
from rankops import _lib  # noqa: E402
lib = _lib.load()
M = 4 * 8 + 4
nwg = ((batch + 63) // 64 + 7) // 8 * 8 * 4  # row tiles rounded to 8, 4 column tiles (n = 512)
buf = (ctypes.c_ulonglong * (nwg * M))()
wbuf = (ctypes.c_uint * (nwg * 4 * 16 * 2))()
lib.rk_debug_lt_phases.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
assert lib.rk_debug_lt_phases(buf, nwg, wbuf) == 0
m = np.array(buf, dtype=np.float64).reshape(nwg, M)
wm = np.array(wbuf, dtype=np.float64).reshape(nwg, 4, 16, 2) / 1e3
live = m[:, 11] > 0
m, wm = m[live], wm[live]


def q(x):
    return f"min {np.min(x):7.2f}  med {np.median(x):7.2f}  max {np.max(x):7.2f}"


print(f"deepfm batch {batch}: graph replay {us:.2f} us (events), {int(live.sum())} live workgroups")
k = m / 1e3
print("prologue        ", q(k[:, 0]), "k cycles")
print("block 0 staged  ", q(k[:, 1]))
for b in range(4):
    print(f"block {b}: mfma issued {q(k[:, 2 + 2 * b])} | barrier {q(k[:, 3 + 2 * b])}")
print("epilogue        ", q(k[:, 10]))
print("end             ", q(k[:, 11]))
w0, w1 = m[:, M - 2], m[:, M - 1]
print("wall: entry spread", q((w0 - w0.min()) / 100), "us; duration", q((w1 - w0) / 100), "us; span",
      f"{(w1.max() - w0.min()) / 100:.2f} us")
print("per wave block 0 issued:", " ".join(f"{v:5.1f}" for v in np.median(wm[:, 1, :, 0], axis=0)))
print("per wave last issued   :", " ".join(f"{v:5.1f}" for v in np.median(wm[:, 0, :, 0], axis=0)))
print("per wave epilogue      :", " ".join(f"{v:5.1f}" for v in np.median(wm[:, 0, :, 1], axis=0)))
