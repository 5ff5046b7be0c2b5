"""Where the DIN headline's short-window overhead goes: samples/s of the prepared configs[2]
forward for timed windows of K = 5 .. 400 steps (bench.py's bracketing: synchronize, perf_counter,
K launches, synchronize; best of 3), and, in one 20-step window, every launch's device duration
and the gaps between launches from HIP events recorded around each launch on the launch stream."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

batch = 4096
model, inp, fn, cfg, _ = bench.workload("din", batch, 0)
run = model.prepare(inp["dense"], inp["category"], inp["sequence"], inp["target"])
for _ in range(20):
    run()
torch.cuda.synchronize()
for K in (5, 10, 20, 50, 100, 400):
    best = 0.0
    for _ in range(3):
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            run()
        torch.cuda.synchronize()
        best = max(best, batch * K / (time.perf_counter() - t0))
    print(f"K={K:4d}: {best / 1e6:6.2f} M samples/s  ({1e6 * batch / best:6.1f} us/step)", flush=True)

st = torch.cuda.current_stream()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
for _ in range(5):
    run()
torch.cuda.synchronize()
t0 = time.perf_counter()
ev[0].record(st)
for k in range(20):
    run()
    ev[k + 1].record(st)
t_issue = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
d = [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(20)]
print("20-step window: host issue %.1f us, wall %.1f us, device (first event -> last) %.1f us"
      % (1e6 * t_issue, 1e6 * t_all, ev[0].elapsed_time(ev[20]) * 1e3))
print("per-launch device time (us):", " ".join(f"{x:.1f}" for x in d))
