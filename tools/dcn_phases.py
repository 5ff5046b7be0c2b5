"""Phase split of the fused MLP kernels (dcn_fused_kernel; MODEL=deepcrossing/bst/deepfm run their
rk_mlp_forward tails) at the bench's batch, from a timing build of the library
(make EXTRA="-DRK_DIN_PHASES -DRK_MLP_PHASES" OUT=../rankops/librankops_phases.so BUILD=build_phases;
point RANKOPS_LIB at it).  Per workgroup, wave 0, cycles from each layer's start to: MFMA loop
issued, epilogue stored (+ next layer's prepare), barrier passed; the stage (prologue) and the
whole workgroup; wall-clock entry/end spread across workgroups.  Marks live in LDS while the
kernel runs and are written out at its end (mlp_core.h RK_MLP_PHASES)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

batch = int(os.environ.get("BATCH", "4096"))
name = os.environ.get("MODEL", "dcn")
model, inp, fn, cfg, _ = bench.workload(name, batch, 0)
g, _ = bench.graph_of(fn)
us = 1e3 * bench.kernel_avg_ms(g.replay)
g.replay()
torch.cuda.synchronize()
from rankops import _lib  # noqa: E402
lib = _lib.load()
M = 4 * 8 + 4
nwg = (batch + 15) // 16
buf = (ctypes.c_ulonglong * (nwg * M))()
wbuf = (ctypes.c_uint * (nwg * 4 * 16 * 2))()
# each kernel module keeps its own counters: the one-launch DeepFM forward reads deepfm_fused.hip's
dbg = lib.rk_debug_deepfm_phases if name == "deepfm" and hasattr(lib, "rk_debug_deepfm_phases") else lib.rk_debug_mlp_phases
dbg.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
assert dbg(buf, nwg, wbuf) == 0
wm = np.array(wbuf, dtype=np.float64).reshape(nwg, 4, 16, 2) / 1e3
m = np.array(buf, dtype=np.float64).reshape(nwg, M)


def q(x):
    return f"min {np.min(x):7.2f}  med {np.median(x):7.2f}  max {np.max(x):7.2f}"


print(f"{name} batch {batch}: graph replay {us:.2f} us (events), {nwg} workgroups")
k = m[:, :M - 2] / 1e3
print("prologue: prepare(0) issued", q(k[:, 28]), "| stage done", q(k[:, 32]), "k cycles")
print("whole workgroup   ", q(k[:, 33]), "k cycles")
for l in range(3):
    print(f"layer {l}: mfma issued {q(k[:, 4*l])} | epilogue {q(k[:, 4*l+1])} | prepare {q(k[:, 4*l+2])} | barrier {q(k[:, 4*l+3])}")
w0, w1 = m[:, M - 2], m[:, M - 1]
print("wall: entry spread", q((w0 - w0.min()) / 100), "us; duration", q((w1 - w0) / 100), "us; span",
      f"{(w1.max() - w0.min()) / 100:.2f} us")
for l in range(3):
    iss = np.median(wm[:, l, :, 0], axis=0)
    epi = np.median(wm[:, l, :, 1], axis=0)
    print(f"layer {l} per wave (median over WGs, k cycles) mfma issued:", " ".join(f"{v:5.1f}" for v in iss))
    print(f"layer {l} per wave                           epilogue   :", " ".join(f"{v:5.1f}" for v in epi))
