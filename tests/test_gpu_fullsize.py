"""Full-size parity: the BASELINE configs that fit one GPU, at their own batch and table sizes,
against the oracle (CPU restatement) run on host copies of the same weights.

  configs[1]  DeepFM, 30 fields x 1,000,000 rows x emb_dim 32, batch 4096   deepfm.py:121-151
  configs[3]  BST, T 64, d_model 128, 4 heads, batch 2048, wechat tables     bst.py:216-247
  configs[4]  DeepFM over 1e8 rows (30 x 3,333,334), ShardedDeepFM at P = 1 on a sampled batch of
              4096, and at P = 8 emulated in one process (tests/a2a_emulator.py) at the real
              per-rank batch 8192 (global 65536)

Tolerance: atol = rtol = 1e-4 (fp32, north star)."""
import gc

import numpy as np
import pytest
import torch

import helpers as H
import rankops
from a2a_emulator import InProcessAllToAll, run_ranks
from oracle import reference_forward as ref
from rankops import sharded

TOL = 1e-4
SHARDED_ROWS = 3_333_334


def _close(got, expect, names, lo=0, hi=None):
    for n, g, e in zip(names, got, expect):
        e = e if hi is None else e[lo:hi]
        torch.testing.assert_close(g.detach().cpu(), e, atol=TOL, rtol=TOL, equal_nan=True,
                                   msg=lambda m: f"{n}: {m}")


def _free():
    gc.collect()
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_configs1_deepfm_full_size():
    cfg = {"dim": 32, "fields": {f"field_{i:02d}": 1_000_000 for i in range(30)}}
    with torch.device("cuda"):
        model = H.build("deepfm", cfg, seed=42)
    model = model.cuda().eval()
    inp = H.to_device(H.make_inputs("deepfm", cfg, 4096, seed=1001), "cuda")
    with torch.no_grad():
        got = model(inp["category"])
        torch.cuda.synchronize()
        p = H.cpu_params(model)
        expect = H.call_oracle("deepfm", cfg, p, H.to_device(inp, "cpu"))
    _close(got, expect, ("prob", "total_logit", "fm1", "fm2", "deep_logit"))
    assert rankops.error_flags() == 0
    del model, p
    _free()


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("pooling", ["sum", "mean"])
def test_configs3_bst_full_size(pooling):
    cfg = {"vocab": H.WECHAT_VOCAB, "T": 64, "dim": 128, "heads": 4, "max_len": 64, "pooling": pooling}
    model = H.build("bst", cfg, seed=42).cuda().eval()
    inp = H.make_inputs("bst", cfg, 2048, seed=1004)
    with torch.no_grad():
        got = model(*[H.to_device(inp[k], "cuda") for k in ("dense", "category", "seq_feedid", "seq_length")])
        torch.cuda.synchronize()
        expect = H.call_oracle("bst", cfg, H.cpu_params(model), inp)
    _close(got, expect, ("prob", "logit"))
    assert rankops.error_flags() == 0


@pytest.fixture(scope="module")
def sharded_1e8():
    """ShardedDeepFM over configs[4]'s 1e8 rows at P = 1 (all 30 fields on this GPU) and host
    copies of its parameters for the oracle."""
    fields = {f"field_{i:02d}": SHARDED_ROWS for i in range(30)}
    torch.manual_seed(42)
    with torch.device("cuda"):
        model = sharded.ShardedDeepFM(fields, 32, [512, 256, 128], rank=0, world_size=1)
    H.randomize_eval_stats(model, 43)
    model.eval()
    p = H.cpu_params(model)
    yield model, fields, p
    del model, p
    _free()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_configs4_sharded_p1_full_tables(sharded_1e8):
    model, fields, p = sharded_1e8
    rng = np.random.default_rng(5000)
    cat = {f: torch.from_numpy(rng.integers(0, SHARDED_ROWS, 4096, dtype=np.int64)) for f in fields}
    with torch.no_grad():
        got = model({f: v.cuda() for f, v in cat.items()})
        torch.cuda.synchronize()
        expect = ref.deepfm_forward(p, cat, list(fields), 3)
    _close(got, expect, ("prob", "total_logit", "fm1", "fm2", "deep_logit"))
    assert rankops.error_flags() == 0


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_configs4_sharded_p8_emulated_full_size(sharded_1e8):
    """configs[4] at full size on one GPU: 8 shards (4/4/4/4/4/4/3/3 fields of 3,333,334 rows),
    local batch 8192 each (global 65536), the chunked exchange pipeline through the emulator."""
    full, fields, p = sharded_1e8
    world, B_l = 8, 8192
    emu = InProcessAllToAll(world)
    shards = []
    for r in range(world):
        sh = sharded.ShardedDeepFM.from_deepfm(full, rank=r, world_size=world)
        sh.exchange_fn = emu.bind(r)
        shards.append(sh)
    assert [len(s.local_fields) for s in shards] == [4, 4, 4, 4, 4, 4, 3, 3]
    rng = np.random.default_rng(6000)
    cat = {f: torch.from_numpy(rng.integers(0, SHARDED_ROWS, world * B_l, dtype=np.int64)) for f in fields}
    dev_cat = {f: v.cuda() for f, v in cat.items()}

    def rank_fn(r):
        with torch.no_grad():
            out = shards[r]({f: v[r * B_l:(r + 1) * B_l] for f, v in dev_cat.items()})
        torch.cuda.synchronize()
        return tuple(o.cpu() for o in out)

    outs = run_ranks(world, rank_fn, on_error=emu.abort)
    assert emu.calls == 1 + 2  # one index exchange, then 2 chunks of 4096 (min_chunk) of rows
    with torch.no_grad():
        expect = ref.deepfm_forward(p, cat, list(fields), 3)
    for r, got in enumerate(outs):
        _close(got, expect, ("prob", "total_logit", "fm1", "fm2", "deep_logit"), r * B_l, (r + 1) * B_l)
    assert rankops.error_flags() == 0
    del shards
    _free()
