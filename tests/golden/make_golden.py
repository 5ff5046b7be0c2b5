"""Generates the golden fixtures tests/golden/<case>.npz from the CPU oracle.

Each fixture holds: the model parameters (reference state_dict keys), the inputs (including
edge cases: empty/full DIN histories, an empty BST sequence), the per-call H2 layers drawn
from torch.manual_seed(meta.draw_seed), and the oracle outputs.  The reference itself cannot
be imported here, so these vectors come from our restatement: they pin the
oracle against regressions and the GPU path against the oracle; they do not pin the oracle
against the reference ("parity unpinned", oracle/__init__.py).

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import helpers as H  # noqa: E402
from oracle import reference_forward as ref  # noqa: E402

SMALL_HIDDEN = [32, 16, 8]
CASES = {
    "dcn": {"hidden": SMALL_HIDDEN, "cross": 2},
    "deepfm": {"hidden": SMALL_HIDDEN, "dim": 8},
    "din": {"hidden": SMALL_HIDDEN, "T": 12},
    "din_softmax": {"hidden": SMALL_HIDDEN, "T": 12, "softmax": True},
    "din_prelu": {"hidden": SMALL_HIDDEN, "T": 5, "activation": "prelu"},
    "afm": {"dim": 8, "att": 16},
    "deepcrossing": {"units": 2, "internal": 16},
    "bst": {"hidden": SMALL_HIDDEN, "T": 10},
    "bst_mean": {"hidden": SMALL_HIDDEN, "T": 10, "pooling": "mean"},
}
B = 16
DRAW_SEED = 7


def model_name(case):
    return case.split("_")[0]


def flatten(prefix, obj, out):
    if isinstance(obj, dict):
        for k, v in obj.items():
            flatten(f"{prefix}::{k}", v, out)
    else:
        out[prefix] = obj.numpy() if isinstance(obj, torch.Tensor) else np.asarray(obj)


def unflatten(arrs, prefix):
    root = {}
    for k, v in arrs.items():
        if not k.startswith(prefix + "::"):
            continue
        parts = k[len(prefix) + 2:].split("::")
        d = root
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = torch.from_numpy(np.array(v))
    return root


def draw_h2(name, cfg, p, inp):
    """Re-draw exactly what the oracle draws per call, in order, from DRAW_SEED."""
    torch.manual_seed(DRAW_SEED)
    if name == "dcn":
        return [t for w, b in ref.draw_cross(50, cfg.get("cross", 1)) for t in (w, b)]
    if name == "din":
        return ref.draw_din_att(p["embeddings.his_read_comment_7d_seq.weight"].shape[1])
    if name == "deepcrossing":
        return [t for _ in range(cfg.get("units", 1)) for t in ref.draw_residual(50, cfg.get("internal", 128))]
    return []


def make(case, cfg):
    name = model_name(case)
    model = H.build(name, cfg, seed=42)
    p = H.cpu_params(model)
    inp = H.make_inputs(name, cfg, B, seed=3000)
    if name == "din":
        lens = inp["sequence"]["his_read_comment_7d_seq_length"]
        lens[0], lens[1], lens[2] = 0, cfg["T"], 1
    if name == "bst":
        inp["seq_length"][0] = 0  # all keys masked -> NaN row (bst.py:80-82)
        inp["seq_length"][1] = cfg["T"]
    torch.manual_seed(DRAW_SEED)
    with torch.no_grad():
        out = H.as_tuple(H.call_oracle(name, cfg, p, inp))
    arrs = {}
    flatten("p", p, arrs)
    flatten("in", inp, arrs)
    for i, o in enumerate(out):
        arrs[f"out::{i}"] = o.numpy() if isinstance(o, torch.Tensor) else np.asarray(o, np.float32)
    for i, t in enumerate(draw_h2(name, cfg, p, inp)):
        arrs[f"h2::{i}"] = t.numpy()
    meta = {"case": case, "model": name, "cfg": cfg, "batch": B, "draw_seed": DRAW_SEED,
            "torch": torch.__version__}
    arrs["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{case}.npz"), **arrs)
    return os.path.getsize(os.path.join(HERE, f"{case}.npz"))


if __name__ == "__main__":
    for case, cfg in CASES.items():
        print(case, make(case, cfg), "bytes")
