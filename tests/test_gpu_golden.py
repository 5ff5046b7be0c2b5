"""GPU path against the committed golden fixtures (parameters + inputs + per-call H2 draws
from a fixed seed + oracle outputs; tests/golden/make_golden.py)."""
import glob
import os

import pytest
import torch

import helpers as H
import rankops
from test_oracle import load_golden

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p)[:-4])
def test_gpu_matches_golden(path):
    meta, p, inp, outs, _ = load_golden(path)
    model = H.build(meta["model"], meta["cfg"], seed=0)
    model.load_state_dict(p, strict=True)
    model = model.cuda().eval()
    torch.manual_seed(meta["draw_seed"])
    with torch.no_grad():
        got = H.as_tuple(H.call_model(model, meta["model"], H.to_device(inp, "cuda")))
    torch.cuda.synchronize()
    assert len(got) == len(outs)
    for g, o in zip(got, outs):
        g = g.detach().cpu() if isinstance(g, torch.Tensor) else torch.tensor(g, dtype=torch.float32)
        torch.testing.assert_close(g.reshape(o.shape), o, atol=1e-4, rtol=1e-4, equal_nan=True)
    assert rankops.error_flags() == 0


@pytest.mark.gpu
def test_reload_and_device_roundtrip_invalidate_caches():
    """load_state_dict and .cpu()/.cuda() round trips must reach the kernels (packed weights,
    folded BatchNorm and [W_q;W_k] caches are rebuilt)."""
    cfg = {"T": 10}
    for name in ("deepfm", "din", "bst"):
        a = H.build(name, cfg, seed=1).cuda()
        b = H.build(name, cfg, seed=2)
        inp = H.to_device(H.make_inputs(name, cfg, 64), "cuda")
        torch.manual_seed(0)
        with torch.no_grad():
            H.call_model(a, name, inp)  # populate caches with seed-1 weights
        a.load_state_dict(b.state_dict())
        torch.manual_seed(0)
        with torch.no_grad():
            got = H.as_tuple(H.call_model(a, name, inp))
        torch.manual_seed(0)
        ref = H.as_tuple(H.call_oracle(name, cfg, H.cpu_params(b), H.to_device(inp, "cpu")))
        torch.testing.assert_close(got[1].cpu(), ref[1], atol=1e-4, rtol=1e-4, equal_nan=True)
        a = a.cpu().cuda()
        torch.manual_seed(0)
        with torch.no_grad():
            got = H.as_tuple(H.call_model(a, name, inp))
        torch.testing.assert_close(got[1].cpu(), ref[1], atol=1e-4, rtol=1e-4, equal_nan=True)
