"""DIN configs[2] forward throughput with S batches in flight: S prepared launches (separate
inputs, outputs and l2 workspaces) issued round-robin on S HIP streams, so one batch's first
workgroups fill the CUs that the previous batch's tail leaves idle.  Prints samples/s for S = 1..4
and checks that every stream's outputs equal its own single-stream launch bit for bit."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402
import helpers as H  # noqa: E402

batch, steps = 4096, int(os.environ.get("STEPS", "400"))
model, inp, fn, cfg, _ = bench.workload("din", batch, 0)
dev = torch.device("cuda", 0)
inps = [inp] + [H.to_device(H.make_inputs("din", cfg, batch, seed=2000 + i), dev) for i in range(3)]
runs = [model.prepare(x["dense"], x["category"], x["sequence"], x["target"]) for x in inps]
ref = []
for r in runs:
    p, lg, l2 = r()
    torch.cuda.synchronize()
    ref.append((p.clone(), lg.clone(), l2.clone() if torch.is_tensor(l2) else l2))
streams = [torch.cuda.Stream() for _ in range(4)]
plans = [r.plan for r in runs]
handles = [st.cuda_stream for st in streams]
# one stream, the default one (as bench.py's single-stream leg)
for n in (50, steps):
    best = 0.0
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            runs[0]()
        torch.cuda.synchronize()
        best = max(best, batch * n / (time.perf_counter() - t0))
    print(f"default stream, {n} steps: {best / 1e6:.2f} M samples/s", flush=True)
for S in (1, 2, 3, 4):
    best = 0.0
    for _ in range(3):
        torch.cuda.synchronize()
        for i in range(S):
            streams[i].wait_stream(torch.cuda.current_stream())
        t0 = time.perf_counter()
        for k in range(steps):
            i = k % S
            plans[i].launch_on(handles[i])
        for i in range(S):
            torch.cuda.current_stream().wait_stream(streams[i])
        torch.cuda.synchronize()
        best = max(best, batch * steps / (time.perf_counter() - t0))
    ok = all(torch.equal(runs[i]()[0], ref[i][0]) for i in range(S))
    torch.cuda.synchronize()
    print(f"S={S}: {best / 1e6:.2f} M samples/s  outputs bit-identical: {ok}", flush=True)
