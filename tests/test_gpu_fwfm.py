"""GPU parity of FwFM (rk_fwfm_forward) against the oracle restatement of FwFM.forward
(oracle/fwfm.py, fwfm.py:114-139): probabilities and logits within 1e-5 / 1e-4 fp32 at the
wechat table sizes, embedding widths on both load paths (16-byte vector and scalar), 2..16
fields, OOB indices, and the LabelEncoder bucketing -> forward chain end to end."""
import numpy as np
import pyarrow as pa
import pytest
import torch

import helpers as H
import rankops
from oracle import fwfm as of
from rankops.fwfm import FwFM

WECHAT_FWFM_DIMS = [H.WECHAT_VOCAB[f] for f in of.FIELDS]  # len(vocab) rows, no +1


def _inputs(dims, B, fields, seed=0):
    g = torch.Generator().manual_seed(seed)
    return {f: torch.randint(0, n, (B,), generator=g) for f, n in zip(fields, dims)}


def _check(m, x_cpu, fields, atol_logit=1e-4):
    p = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    want_p, want_y = of.forward(p, x_cpu, fields)
    prob, logit = m({f: t.cuda() for f, t in x_cpu.items()}, return_logit=True)
    torch.cuda.synchronize()
    torch.testing.assert_close(logit.cpu(), want_y, rtol=0, atol=atol_logit)
    torch.testing.assert_close(prob.cpu(), want_p, rtol=0, atol=1e-5)
    prob2 = m({f: t.cuda() for f, t in x_cpu.items()})
    assert prob2.shape == want_p.shape
    torch.testing.assert_close(prob2.cpu(), want_p, rtol=0, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 7, 4096, 65537])
def test_fwfm_wechat_default(B):
    torch.manual_seed(0)
    m = FwFM(WECHAT_FWFM_DIMS, 8).cuda().eval()
    _check(m, _inputs(WECHAT_FWFM_DIMS, B, of.FIELDS), of.FIELDS)
    assert rankops.error_flags() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [1, 3, 4, 5, 12, 16, 33, 64, 100, 256])
def test_fwfm_embedding_widths(dim):
    torch.manual_seed(1)
    dims = [50, 70, 2, 40, 30, 60]
    m = FwFM(dims, dim).cuda().eval()
    _check(m, _inputs(dims, 1000, of.FIELDS, seed=dim), of.FIELDS, atol_logit=2e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("F", [2, 3, 9, 16])
def test_fwfm_field_counts(F):
    torch.manual_seed(2)
    fields = tuple(f"field_{i}" for i in range(F))
    dims = [11 + 3 * i for i in range(F)]
    m = FwFM(dims, 8, field_names=fields).cuda().eval()
    _check(m, _inputs(dims, 513, fields, seed=F), fields)


@pytest.mark.gpu
def test_fwfm_unsupported_field_count_fails_loudly():
    fields = tuple(f"field_{i}" for i in range(17))
    m = FwFM([5] * 17, 8, field_names=fields).cuda().eval()
    with pytest.raises(rankops.RankOpsError):
        m({f: torch.zeros(4, dtype=torch.long, device="cuda") for f in fields})


@pytest.mark.gpu
def test_fwfm_oob_index_flagged():
    m = FwFM([5, 5, 5, 5, 5, 5], 8).cuda().eval()
    rankops.error_flags()
    x = {f: torch.zeros(4, dtype=torch.long, device="cuda") for f in of.FIELDS}
    x["feedid"][2] = 5
    m(x)
    torch.cuda.synchronize()
    assert rankops.error_flags() != 0


@pytest.mark.gpu
def test_fwfm_label_encode_to_forward():
    """Raw string columns -> rankops.label_encode -> FwFM on the GPU, against the oracle chain."""
    rng = np.random.default_rng(5)
    vocabs = {f: [f"{f}_{i}" for i in rng.permutation(2 * n)[:n]] for f, n in zip(of.FIELDS, [97, 131, 2, 53, 61, 47])}
    cols = {}
    for f, v in vocabs.items():
        vals = [v[i] for i in rng.integers(0, len(v), 3000)]
        vals[:40] = [v[0]] * 40  # a clear mode
        for i in rng.integers(40, 3000, 100):
            vals[i] = None if i % 2 else f"{f}_oov"
        cols[f] = vals
    dims = [len(vocabs[f]) for f in of.FIELDS]
    torch.manual_seed(4)
    m = FwFM(dims, 8).cuda().eval()
    x = {}
    for f in of.FIELDS:
        voc = rankops.Vocabulary(text="".join(w + "\n" for w in vocabs[f]).encode())
        enc = rankops.label_encode(pa.array(cols[f]), voc)
        want = of.encode_column(cols[f], vocabs[f])
        np.testing.assert_array_equal(enc, want)
        x[f] = torch.from_numpy(enc)
    _check(m, x, of.FIELDS)


def _train_check(dims, D, fields, B, seed, steps=2):
    """FwFM train steps (fwfm.py:141-160: forward, BCELoss, backward, Adam) against the oracle
    forward differentiated by autograd; gradients within 5e-4 of each tensor's largest."""
    torch.manual_seed(seed)
    m = FwFM(dims, D, field_names=fields).cuda().train()
    x = _inputs(dims, B, fields, seed=seed)
    label = (torch.rand(B, generator=torch.Generator().manual_seed(seed)) < 0.3).float()
    params = dict(m.named_parameters())
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    opt = rankops.Adam(m.parameters(), lr=1e-3)
    ref_opt = torch.optim.Adam([p[n] for n in params], lr=1e-3)
    crit = torch.nn.BCELoss()
    xd = {f: t.cuda() for f, t in x.items()}
    for step in range(steps):
        opt.zero_grad()
        ref_opt.zero_grad()
        prob = m(xd)
        crit(prob, label.cuda()).backward()
        want, _ = of.forward(p, x, fields)
        crit(want, label).backward()
        torch.testing.assert_close(prob.detach().cpu(), want.detach(), rtol=0, atol=1e-5)
        for n, prm in params.items():
            scale = max(1e-4, float(p[n].grad.abs().max()))
            torch.testing.assert_close(prm.grad.cpu(), p[n].grad, rtol=0, atol=5e-4 * scale,
                                       msg=lambda msg: f"grad {n} step {step}: {msg}")
        opt.step()
        ref_opt.step()
        for n, prm in params.items():
            torch.testing.assert_close(prm.detach().cpu(), p[n].detach(), rtol=1e-4, atol=2e-5,
                                       msg=lambda msg: f"param {n} step {step}: {msg}")
        with torch.no_grad():  # re-synchronise (Adam's sign flips on noise-level gradients)
            for n, prm in params.items():
                p[n].copy_(prm.detach().cpu())
                for key in ("exp_avg", "exp_avg_sq"):
                    ref_opt.state[p[n]][key].copy_(opt.state[prm][key].cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("D", [8, 5, 32])
def test_fwfm_train_steps_match_autograd(D):
    _train_check([50, 70, 2, 40, 30, 60], D, of.FIELDS, 1024, seed=D)


@pytest.mark.gpu
def test_fwfm_train_wechat_and_16_fields():
    _train_check(WECHAT_FWFM_DIMS, 8, of.FIELDS, 4096, seed=3, steps=1)
    fields = tuple(f"field_{i}" for i in range(16))
    _train_check([11 + 3 * i for i in range(16)], 16, fields, 777, seed=4)
