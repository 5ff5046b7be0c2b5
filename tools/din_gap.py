"""Graph replays of the DIN eval forward (configs[2] shape; DIN_T overrides the history length,
BATCH the batch): prints us/step, and under rocprofv3 --kernel-trace gives the kernel durations
and gaps (tools/trace_gaps.py).  RANKOPS_DIN_BALANCE=0/1 selects the workgroup assignment."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import bench  # noqa: E402
import helpers as H  # noqa: E402
import torch  # noqa: E402

T = int(os.environ.get("DIN_T", "50"))
B = int(os.environ.get("BATCH", "4096"))
cfg = {"vocab": H.WECHAT_VOCAB, "T": T, "dim": 32, "interaction_weights": "frozen"}
dev = torch.device("cuda", 0)
with torch.device(dev):
    model = H.build("din", cfg, seed=42)
model = model.to(dev).eval()
inp = H.to_device(H.make_inputs("din", cfg, B, seed=1000), dev)
g, out = bench.graph_of(lambda: H.call_model(model, "din", inp))
for _ in range(50):
    g.replay()
torch.cuda.synchronize()
best = 1e9
for _ in range(3):
    t0 = time.perf_counter()
    for _ in range(300):
        g.replay()
    torch.cuda.synchronize()
    best = min(best, (time.perf_counter() - t0) / 300)
print(f"T={T} B={B} balance={os.environ.get('RANKOPS_DIN_BALANCE', 'auto')}: {1e6 * best:.2f} us/step "
      f"({B / best / 1e6:.2f} M samples/s)")
