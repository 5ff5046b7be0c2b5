"""Host-side cost of the eager paths (the reference's loops call the model eagerly, dcn.py:188-239):
cProfile of N eager eval forwards and N eager train steps per model, top functions by own time.
    python tools/host_profile.py [models] [N]"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

models = (sys.argv[1] if len(sys.argv) > 1 else "dcn,deepfm,fwfm,din,bst").split(",")
N = int(sys.argv[2]) if len(sys.argv) > 2 else 50


def eval_step(name):
    model, inp, fn, cfg, _ = bench.workload(name, 2048 if name == "bst" else 4096, 0)

    def run():
        with torch.no_grad():
            fn()
    return run


def train_step(name):
    import helpers as H
    import rankops
    cfg = {"dcn": {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen"},
           "deepfm": {"vocab": H.WECHAT_VOCAB}, "fwfm": {"vocab": H.WECHAT_VOCAB, "dim": 8},
           "din": {"vocab": H.WECHAT_VOCAB, "T": 50, "dim": 32, "interaction_weights": "frozen"},
           "bst": {"vocab": H.WECHAT_VOCAB, "T": 64, "dim": 128, "heads": 4, "max_len": 64}}[name]
    batch = 2048 if name == "bst" else 4096
    model = H.build(name, cfg).cuda().train()
    inp = H.to_device(H.make_inputs(name, cfg, batch, seed=77), "cuda")
    label = (torch.rand(batch, device="cuda") < 0.3).float()
    on_logit = name in ("dcn", "bst")
    crit = torch.nn.BCEWithLogitsLoss() if on_logit else torch.nn.BCELoss()
    opt = rankops.Adam(model.parameters(), lr=1e-3)

    def run():
        opt.zero_grad(set_to_none=True)
        out = H.as_tuple(H.call_model(model, name, inp))
        loss = crit(out[1].squeeze(), label) if on_logit else crit(out[0].squeeze(), label)
        if name == "din":
            loss = loss + out[2]
        loss.backward()
        opt.step()
    return run


kinds = os.environ.get("KINDS", "eval,train").split(",")
# run the autograd backward on this thread, so that cProfile sees the HIP backward's host side
torch.autograd.set_multithreading_enabled(False)
for name in models:
    for kind, mk in (("eval", eval_step), ("train", train_step)):
        if kind not in kinds:
            continue
        run = mk(name)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(N):
            run()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / N
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(N):
            run()
        pr.disable()
        torch.cuda.synchronize()
        s = io.StringIO()
        st = pstats.Stats(pr, stream=s)
        st.sort_stats(os.environ.get("SORT", "tottime")).print_stats(int(os.environ.get("LINES", "14")))
        print(f"===== {name} {kind}: eager {1e3 * wall:.3f} ms/step")
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        print("\n".join(line.replace(root + "/", "") for line in s.getvalue().splitlines()[4:60]))
