"""Eager vs hipGraph training step (bench.bench_train) for a few models, steps x repeats:
    python tools/train_ratio.py [models] [steps] [repeats]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

models = (sys.argv[1] if len(sys.argv) > 1 else "dcn,fwfm,deepfm").split(",")
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
for m in models:
    for _ in range(reps):
        r = bench.bench_train(2048 if m == "bst" else 4096, steps, 10, m)
        e, g = r["eager"]["ms_per_step"], r["graph"]["ms_per_step"]
        print(f"{m:8s} eager {e:.4f} ms  graph {g:.4f} ms  ratio {e / g:.2f}", flush=True)
