"""Host floor of an eager training step: the reference loop's structure —
zero_grad, a forward through one autograd Function over all the model's parameters, the script's
loss, loss.backward(), rankops.Adam — with a Function that launches nothing (outputs and
gradients are torch.empty), against the real eager step and its hipGraph replay.
    python tools/train_floor.py [models] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

import helpers as H  # noqa: E402
import rankops  # noqa: E402


class _Null(torch.autograd.Function):
    @staticmethod
    def forward(ctx, B, *params):
        ctx.shapes = [p.shape for p in params]
        dev = params[0].device
        return torch.empty(B, device=dev), torch.empty(B, device=dev)

    @staticmethod
    def backward(ctx, dprob, dlogit):
        # gradients carved from one flat buffer, as rankops' own backward does (train.zero_grads)
        # minus its fill: the allocator hands the same block back every step, so rankops.Adam's
        # cached argument block stays valid
        dev = dprob.device
        sizes = [(int(torch.Size(s).numel()) + 63) // 64 * 64 for s in ctx.shapes]
        flat = torch.empty(sum(sizes), device=dev)
        out, off = [], 0
        for s, n in zip(ctx.shapes, sizes):
            out.append(flat[off:off + torch.Size(s).numel()].view(s))
            off += n
        return (None, *out)


models = (sys.argv[1] if len(sys.argv) > 1 else "dcn,fwfm,deepfm").split(",")
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
for name in models:
    cfg = {"dcn": {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen"}, "deepfm": {"vocab": H.WECHAT_VOCAB},
           "fwfm": {"vocab": H.WECHAT_VOCAB, "dim": 8}}[name]
    batch = 4096
    model = H.build(name, cfg).cuda().train()
    params = list(model.parameters())
    label = (torch.rand(batch, device="cuda") < 0.3).float()
    on_logit = name == "dcn"
    crit = torch.nn.BCEWithLogitsLoss() if on_logit else torch.nn.BCELoss()
    opt = rankops.Adam(params, lr=1e-3)

    def step():
        opt.zero_grad(set_to_none=True)
        prob, logit = _Null.apply(batch, *params)
        loss = crit(logit, label) if on_logit else crit(prob.sigmoid(), label)
        loss.backward()
        opt.step()

    for _ in range(20):
        step()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / steps)
    real = bench.bench_train(batch, 60, 10, name)
    print(f"{name:8s} floor {1e3 * best:.4f} ms  eager {real['eager']['ms_per_step']:.4f} ms  "
          f"graph {real['graph']['ms_per_step']:.4f} ms  ({len(params)} parameters)", flush=True)
