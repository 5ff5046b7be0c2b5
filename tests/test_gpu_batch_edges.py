"""GPU: the batch-size edges of every model's eval forward through the HIP path — an empty batch
(B = 0: the reference's torch ops return empty outputs of the right shape, and so must the engine,
launching nothing that reads past the inputs), a single sample, and a batch one past a 16-row
workgroup and one past a full 256-CU wave of them (ragged last tiles) — against the oracle on the
same seeded inputs (atol/rtol 1e-4, the north star's fp32 tolerance)."""
import pytest
import torch

import helpers as H
import rankops

ATOL = RTOL = 1e-4

MODELS = [
    ("dcn", {}),
    ("deepfm", {}),
    ("din", {"T": 50, "interaction_weights": "frozen"}),
    ("afm", {}),
    ("deepcrossing", {}),
    ("bst", {"T": 50}),
    ("bst", {"T": 64, "dim": 128, "max_len": 64}),
    ("fwfm", {}),
]


def _ids(c):
    return c[0] + ("-" + "-".join(f"{k}{v}" for k, v in c[1].items()) if c[1] else "")


@pytest.mark.gpu
@pytest.mark.parametrize("case", MODELS, ids=_ids)
def test_empty_batch(case):
    name, cfg = case
    model = H.build(name, cfg).cuda().eval()
    inp = H.to_device(H.make_inputs(name, cfg, 0), "cuda")
    rankops.error_flags(reset=True)
    with torch.no_grad():
        out = H.as_tuple(H.call_model(model, name, inp))
    torch.cuda.synchronize()
    for o in out:
        if isinstance(o, torch.Tensor) and o.dim() > 0:
            assert o.shape[0] == 0, (name, tuple(o.shape))
    assert rankops.error_flags() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("edge", ["one", "tile_plus_one", "wave_plus_one"])
@pytest.mark.parametrize("case", [c for c in MODELS if c[0] != "fwfm"], ids=_ids)  # FwFM: test_gpu_fwfm.py
def test_ragged_batches_against_oracle(case, edge):
    name, cfg = case
    # d 128 BST: its persistent kernel walks samples b + k * 256, so 257 is its wave edge (and keeps
    # the CPU oracle's transformer to seconds)
    wave = 257 if cfg.get("dim") == 128 else 4097
    B = {"one": 1, "tile_plus_one": 17, "wave_plus_one": wave}[edge]
    if name == "din":
        cfg = {k: v for k, v in cfg.items() if k != "interaction_weights"}  # per-call draws: seeded below
    model = H.build(name, cfg)
    inp = H.make_inputs(name, cfg, B, seed=B + 7)
    torch.manual_seed(123)
    with torch.no_grad():
        ref = H.as_tuple(H.call_oracle(name, cfg, H.cpu_params(model), inp))
    model = model.cuda().eval()
    torch.manual_seed(123)
    with torch.no_grad():
        out = H.as_tuple(H.call_model(model, name, H.to_device(inp, "cuda")))
    torch.cuda.synchronize()
    assert len(out) == len(ref)
    for o, r in zip(out, ref):
        if isinstance(r, torch.Tensor):
            torch.testing.assert_close(o.cpu().reshape(r.shape), r, atol=ATOL, rtol=RTOL, equal_nan=True)
    assert rankops.error_flags() == 0
