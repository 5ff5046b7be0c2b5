"""Shader clock inside gemm_rows_kernel under its own load (timing build: make EXTRA=-DRK_ROWS_CLOCK
OUT=<lib> BUILD=build_clk; RANKOPS_LIB=<lib>): per workgroup clock64 and wall-clock (100 MHz) deltas
of one launch at the BST training shape -> effective MHz, and the MFMA-busy fraction at that clock."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd")
import rankops  # noqa: E402
from rankops import _lib, ops  # noqa: E402

rankops.load_library()
lib = _lib.load()
M, N, K = int(os.environ.get("M", "131072")), 128, 128
x = torch.randn(M, K, device="cuda")
w = torch.randn(N, K, device="cuda")
b = torch.randn(N, device="cuda")
y = torch.empty(M, N, device="cuda")
ep = ops.make_epilogue(bias=b, act="relu")
for _ in range(30):
    ops.linear(x, w, y, epilogue=ep)
torch.cuda.synchronize()
ops.linear(x, w, y, epilogue=ep)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (4096 * 4))()
lib.rk_debug_rows_clock.argtypes = [ctypes.c_void_p]
assert lib.rk_debug_rows_clock(buf) == 0
a = np.array(buf, dtype=np.float64).reshape(4096, 4)
a = a[a[:, 3] > 0]
cyc = a[:, 1] - a[:, 0]
wall_us = (a[:, 3] - a[:, 2]) / 100.0
mhz = cyc / wall_us
span_us = (a[:, 3].max() - a[:, 2].min()) / 100.0
# MFMA work per workgroup: 4 waves x slabs x 16 chunks x 16 v_mfma_f32_32x32x2 (64 cycles) on 4 SIMDs
nwg = len(a)
slabs_per_wave = (M / 32) / (nwg * 4)
mfma_cyc_per_simd = slabs_per_wave * 16 * 16 * 64 * 2  # 2 workgroups per CU share the SIMDs
print(f"{nwg} workgroups, kernel span {span_us:.1f} us; per-WG wall med {np.median(wall_us):.1f} us; "
      f"shader clock med {np.median(mhz):.0f} MHz (min {mhz.min():.0f} max {mhz.max():.0f})")
print(f"MFMA cycles per SIMD {mfma_cyc_per_simd:.0f} = {mfma_cyc_per_simd / np.median(mhz):.1f} us at that clock "
      f"-> busy {mfma_cyc_per_simd / np.median(mhz) / np.median(wall_us):.2f} of the workgroup's wall time")
st = (a[:, 2] - a[:, 2].min()) / 100.0
en = (a[:, 3] - a[:, 2].min()) / 100.0
q = lambda v: f"min {v.min():6.1f} med {np.median(v):6.1f} max {v.max():6.1f}"  # noqa: E731
print("start offset us:", q(st), "| end offset us:", q(en))
order = np.argsort(st)
print("start offset by dispatch order (every 64th WG):", " ".join(f"{st[i]:.1f}" for i in range(0, nwg, 64)))
