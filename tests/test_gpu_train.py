"""GPU parity of the training path: each backward kernel against torch
autograd in fp32/fp64 on the CPU, rankops.Adam against torch.optim.Adam, and whole DCN train
steps (forward, loss.backward(), optimizer.step()) against the oracle restatement of
DCNModel.forward (oracle/reference_forward.py, dcn.py:161-180) differentiated by autograd —
the reference's own training mechanism.  Tolerances are written per test."""
import numpy as np
import pytest
import torch

import helpers as H
import rankops
from oracle import reference_forward as ref
from rankops import ops


def _gemm_case(TA, TB, M, N, R, masked, seed):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn((R, M) if TA else (M, R), generator=g)
    B = torch.randn((R, N) if TB else (N, R), generator=g)
    mask = (torch.rand(A.shape, generator=g) > 0.4).float() * torch.rand(A.shape, generator=g) if masked else None
    opA = (A.t() if TA else A).double()
    if masked:
        opA = opA * ((mask.t() if TA else mask) > 0).double()
    opB = (B.t() if TB else B).double()
    return A, B, mask, opA @ opB.t(), opA.sum(1)


@pytest.mark.gpu
@pytest.mark.parametrize("TA", [0, 1])
@pytest.mark.parametrize("TB", [0, 1])
@pytest.mark.parametrize("shape", [(1, 1, 1), (64, 64, 32), (100, 70, 33), (4096, 50, 512), (512, 48, 4096),
                                   (3, 300, 1000)])
@pytest.mark.parametrize("split", [0, 1, 3])
def test_gemm_matches_fp64(TA, TB, shape, split):
    M, N, R = shape
    A, B, mask, want, rs = _gemm_case(TA, TB, M, N, R, masked=(M + N) % 2 == 0, seed=M * 7 + N + R)
    C = torch.full((M, N), 7.0, device="cuda")
    sums = torch.full((M,), 7.0, device="cuda")
    Ad, Bd = A.cuda(), B.cuda()
    ops.gemm(TA, TB, M, N, R, Ad, Ad.stride(0), Bd, Bd.stride(0), C, A_mask=mask.cuda() if mask is not None else None,
             row_sums=sums, split=split)
    tol = 1e-4 * max(1.0, float(want.abs().max()))
    torch.testing.assert_close(C.cpu().double(), want, rtol=0, atol=tol)
    torch.testing.assert_close(sums.cpu().double(), rs, rtol=0, atol=tol)
    # accumulate adds on top
    ops.gemm(TA, TB, M, N, R, Ad, Ad.stride(0), Bd, Bd.stride(0), C, A_mask=mask.cuda() if mask is not None else None,
             accumulate=True, split=split)
    torch.testing.assert_close(C.cpu().double(), 2 * want, rtol=0, atol=2 * tol)


@pytest.mark.gpu
def test_gemm_strided_output():
    A, B, _, want, _ = _gemm_case(0, 1, 37, 20, 45, False, 1)
    C = torch.zeros(37, 64, device="cuda")
    ops.gemm(False, True, 37, 20, 45, A.cuda(), 45, B.cuda(), 20, C, 64)
    torch.testing.assert_close(C[:, :20].cpu().double(), want, rtol=0, atol=1e-4)
    assert float(C[:, 20:].abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,K", [(4096, 512, 50), (1000, 256, 512), (7, 128, 256)])
def test_linear_relu_backward(B, N, K):
    g = torch.Generator().manual_seed(B + N)
    x = torch.randn(B, K, generator=g)
    lin = torch.nn.Linear(K, N)
    xr = x.clone().requires_grad_(True)
    y = torch.relu(lin(xr))
    dy = torch.randn(B, N, generator=g)
    y.backward(dy)
    h = y.detach().cuda()
    dx, dW, db = ops.linear_backward(dy.cuda(), x.cuda(), lin.weight.detach().cuda(), relu_out=h)
    torch.testing.assert_close(dx.cpu(), xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dW.cpu(), lin.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db.cpu(), lin.bias.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("ka,kb", [(50, 128), (50, 300), (7, 0)])
def test_logit_head_backward(ka, kb):
    B = 1000
    g = torch.Generator().manual_seed(ka + kb)
    xa, xb = torch.randn(B, ka, generator=g), torch.randn(B, kb, generator=g)
    lin = torch.nn.Linear(ka + kb, 1)
    xa_r, xb_r = xa.clone().requires_grad_(True), xb.clone().requires_grad_(True)
    logit = lin(torch.cat([xa_r, xb_r], 1))
    prob = torch.sigmoid(logit)
    dlogit, dprob = torch.randn(B, 1, generator=g), torch.randn(B, 1, generator=g)
    torch.autograd.backward([logit, prob], [dlogit, dprob])
    dev = "cuda"
    dxa, dxb = torch.empty(B, ka, device=dev), torch.empty(B, kb, device=dev)
    dw, db = torch.empty(1, ka + kb, device=dev), torch.empty(1, device=dev)
    ops.logit_head_backward(dlogit.cuda(), dprob.cuda(), prob.detach().cuda(), xa.cuda(),
                            xb.cuda() if kb else None, lin.weight.detach().cuda(), dxa, dxb if kb else None, dw, db)
    torch.testing.assert_close(dxa.cpu(), xa_r.grad, rtol=1e-5, atol=1e-5)
    if kb:
        torch.testing.assert_close(dxb.cpu(), xb_r.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dw.cpu(), lin.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db.cpu(), lin.bias.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("L,d", [(1, 50), (3, 50), (0, 50), (8, 200)])
def test_dcn_cross_backward(L, d):
    B = 513
    g = torch.Generator().manual_seed(L * 100 + d)
    x0 = torch.randn(B, d, generator=g)
    cw, cb = torch.randn(L, d, generator=g) * 0.2, torch.randn(L, d, generator=g) * 0.1
    x0r = x0.double().requires_grad_(True)  # fp64 reference: deep stacks amplify fp32 rounding
    xl = x0r
    for l in range(L):
        xl = ref.dcn_cross_layer(x0r, xl, cw[l].double().reshape(d, 1), cb[l].double().reshape(d, 1))
    dxl = torch.randn(B, d, generator=g)
    xl.backward(dxl.double())
    base = torch.randn(B, d, generator=g)
    dx0 = base.clone().cuda()
    ops.dcn_cross_backward(x0.cuda(), cw.cuda(), cb.cuda(), L, dxl.cuda(), dx0, accumulate=True)
    want = base.double() + x0r.grad
    torch.testing.assert_close(dx0.cpu().double(), want, rtol=1e-4, atol=1e-5 * float(want.abs().max()))


@pytest.mark.gpu
def test_embedding_backward_dense_grad():
    B, W = 4096, 30
    g = torch.Generator().manual_seed(3)
    dx = torch.randn(B, W, generator=g)
    rows = [5, 1000, 2]
    idx = [torch.randint(0, r, (B,), generator=g) for r in rows]
    idx[0][:100] = 3  # a hot row
    grads = [torch.zeros(r, d, device="cuda") for r, d in zip(rows, (4, 16, 2))]
    dxd = dx.cuda()
    idx_d = [i.cuda() for i in idx]  # segments hold raw pointers: keep the tensors alive
    segs = [ops.dense_segment(dxd, 8, 0)]
    col = 8
    for gr, i in zip(grads, idx_d):
        segs.append(ops.table_segment(gr, i, col))
        col += gr.shape[1]
    ops.embedding_backward(segs, B, dxd)
    col = 8
    for gr, i in zip(grads, idx):
        want = torch.zeros(gr.shape).index_add_(0, i, dx[:, col:col + gr.shape[1]])
        torch.testing.assert_close(gr.cpu(), want, rtol=1e-5, atol=1e-4)
        col += gr.shape[1]


@pytest.mark.gpu
@pytest.mark.parametrize("n,rows,dim", [(131072, 106445, 128), (204800, 106445, 32), (1000, 7, 5), (1, 3, 4)])
def test_embedding_backward_sorted_matches_index_add(n, rows, dim):
    """Sorted segment-reduce scatter against index_add_ (fp64) with half the ids on one hot row,
    a strided dx segment and out-of-range ids (skipped, flagged)."""
    g = torch.Generator().manual_seed(n + dim)
    idx = torch.randint(0, rows, (n,), generator=g)
    idx[::2] = 0  # padded history positions
    ld = dim + 3
    dx = torch.randn(n, ld, generator=g)
    grad = torch.zeros(rows, dim, device="cuda")
    rankops.error_flags(reset=True)
    idx_d, dx_d = idx.cuda(), dx.cuda()
    ops.embedding_backward_sorted(ops.table_segment(grad, idx_d, 2), n, dx_d)
    want = torch.zeros(rows, dim, dtype=torch.float64).index_add_(0, idx, dx[:, 2:2 + dim].double())
    torch.testing.assert_close(grad.cpu().double(), want, rtol=1e-5, atol=1e-4 * max(1.0, float(want.abs().max())))
    assert rankops.error_flags() == 0
    if n > 4:
        bad = idx.clone()
        bad[3] = rows + 5
        bad[4] = -1
        grad.zero_()
        bad_d = bad.cuda()
        ops.embedding_backward_sorted(ops.table_segment(grad, bad_d, 2), n, dx_d)
        keep = (bad >= 0) & (bad < rows)
        want = torch.zeros(rows, dim, dtype=torch.float64).index_add_(0, bad[keep], dx[keep, 2:2 + dim].double())
        torch.testing.assert_close(grad.cpu().double(), want, rtol=1e-5, atol=1e-4 * max(1.0, float(want.abs().max())))
        assert rankops.error_flags(reset=True) & 1


@pytest.mark.gpu
@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_adam_matches_torch(wd):
    g = torch.Generator().manual_seed(11)
    shapes = [(1000, 16), (3,), (512, 50), (1,), (70000,)]
    ps = [torch.randn(s, generator=g).cuda() for s in shapes]
    qs = [p.clone() for p in ps]
    pa = [torch.nn.Parameter(p) for p in ps]
    qa = [torch.nn.Parameter(q) for q in qs]
    ours = rankops.Adam(pa, lr=3e-3, weight_decay=wd)
    theirs = torch.optim.Adam(qa, lr=3e-3, weight_decay=wd)
    for step in range(6):
        for a, b in zip(pa, qa):
            gr = torch.randn(a.shape, generator=g).cuda() * (step + 1)
            a.grad, b.grad = gr.clone(), gr.clone()
        if step == 3:
            pa[1].grad = None  # a parameter that skips a step keeps its own step count
            qa[1].grad = None
        ours.step()
        theirs.step()
    for a, b in zip(pa, qa):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-6, atol=1e-6)
    for a, b in zip(pa, qa):
        sa, sb = ours.state[a], theirs.state[b]
        assert float(sa["step"]) == float(sb["step"])
        # a few elements differ by an ulp (fma contraction of the lerp / addcmul)
        torch.testing.assert_close(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-6)
    # state dicts are interchangeable with torch.optim.Adam
    ours2 = rankops.Adam(pa, lr=3e-3, weight_decay=wd)
    ours2.load_state_dict(theirs.state_dict())
    assert float(ours2.state[pa[0]]["step"]) == 6.0


def _dcn_oracle_params(model):
    return {k: v.detach().cpu().clone().requires_grad_(True) for k, v in model.state_dict().items()}


def _dcn_step_check(model, cfg, B, seed, steps, opt_kind):
    inp = H.make_inputs("dcn", cfg, B, seed=seed)
    label = (torch.rand(B, generator=torch.Generator().manual_seed(seed)) < 0.3).float()
    p = _dcn_oracle_params(model)
    names = [n for n, _ in model.named_parameters()]
    opt = rankops.Adam(model.parameters(), lr=1e-3) if opt_kind == "rankops" else \
        torch.optim.Adam(model.parameters(), lr=1e-3)
    ref_opt = torch.optim.Adam([p[n] for n in names], lr=1e-3)
    crit = torch.nn.BCEWithLogitsLoss()
    dinp = H.to_device(inp, "cuda")
    hidden = len(cfg.get("hidden", [512, 256, 128]))
    L = cfg.get("cross", 1)
    for step in range(steps):
        opt.zero_grad()
        ref_opt.zero_grad()
        torch.manual_seed(1234 + step)  # per-call cross draws: same generator state on both sides
        prob, logit = H.call_model(model, "dcn", dinp)
        loss = crit(logit.squeeze(), label.cuda())
        loss.backward()
        torch.manual_seed(1234 + step)
        rprob, rlogit = ref.dcn_forward(p, inp["dense"], inp["category"], L, hidden)
        rloss = crit(rlogit.squeeze(), label)
        rloss.backward()
        torch.testing.assert_close(logit.detach().cpu(), rlogit.detach(), rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(prob.detach().cpu(), rprob.detach(), rtol=1e-4, atol=1e-4)
        assert abs(float(loss.detach()) - float(rloss.detach())) < 1e-5
        for n, prm in model.named_parameters():
            want = p[n].grad
            scale = max(1e-3, float(want.abs().max()))
            torch.testing.assert_close(prm.grad.cpu(), want, rtol=0, atol=2e-4 * scale, msg=f"grad {n} step {step}")
        opt.step()
        ref_opt.step()
        for n, prm in model.named_parameters():
            torch.testing.assert_close(prm.detach().cpu(), p[n].detach(), rtol=1e-4, atol=1e-5,
                                       msg=f"param {n} after step {step}")


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{}, {"cross": 3}, {"cross": 0}, {"hidden": [64, 300]}, {"vocab": H.WECHAT_VOCAB}],
                         ids=["default", "cross3", "cross0", "wide_last", "wechat"])
def test_dcn_train_steps_match_autograd(cfg):
    model = H.build("dcn", cfg).cuda().train()
    _dcn_step_check(model, cfg, 1024, seed=2000, steps=3, opt_kind="rankops")


@pytest.mark.gpu
def test_dcn_train_with_torch_adam_and_eval_after():
    """The reference loop unchanged (torch.optim.Adam), then eval forward on the updated weights."""
    model = H.build("dcn", {}).cuda().train()
    _dcn_step_check(model, {}, 512, seed=2100, steps=2, opt_kind="torch")
    model.eval()
    inp = H.to_device(H.make_inputs("dcn", {}, 64, seed=5), "cuda")
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    torch.manual_seed(9)
    with torch.no_grad():
        prob, logit = H.call_model(model, "dcn", inp)
    torch.manual_seed(9)
    rprob, rlogit = ref.dcn_forward(p, H.to_device(inp, "cpu")["dense"], H.to_device(inp, "cpu")["category"], 1, 3)
    torch.testing.assert_close(logit.cpu(), rlogit, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_dcn_train_no_grad_is_forward_only():
    model = H.build("dcn", {"interaction_weights": "frozen"}).cuda().train()
    inp = H.to_device(H.make_inputs("dcn", {}, 32), "cuda")
    with torch.no_grad():
        prob, logit = H.call_model(model, "dcn", inp)
    assert not prob.requires_grad
    prob2, logit2 = H.call_model(model, "dcn", inp)
    assert prob2.requires_grad
    torch.testing.assert_close(prob2.detach(), prob)


@pytest.mark.gpu
def test_adam_capturable_matches_torch_capturable():
    g = torch.Generator().manual_seed(12)
    shapes = [(1000, 16), (3,), (70000,)]
    pa = [torch.nn.Parameter(torch.randn(s, generator=g).cuda()) for s in shapes]
    qa = [torch.nn.Parameter(p.detach().clone()) for p in pa]
    ours = rankops.Adam(pa, lr=2e-3, capturable=True)
    theirs = torch.optim.Adam(qa, lr=2e-3, capturable=True)
    for step in range(5):
        for a, b in zip(pa, qa):
            gr = torch.randn(a.shape, generator=g).cuda()
            a.grad, b.grad = gr.clone(), gr.clone()
        ours.step()
        theirs.step()
    for a, b in zip(pa, qa):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-6, atol=1e-6)
        assert ours.state[a]["step"].device.type == "cuda" and float(ours.state[a]["step"]) == 5.0


@pytest.mark.gpu
def test_dcn_train_step_graph_capture_matches_eager():
    """Whole train step (zero_grad, forward, loss.backward(), capturable rankops.Adam) captured in
    one hipGraph and replayed, against the same steps run eagerly on a twin model."""
    cfg = {"interaction_weights": "frozen"}
    B = 512
    a = H.build("dcn", cfg).cuda().train()
    b = H.build("dcn", cfg).cuda().train()
    b.load_state_dict(a.state_dict())
    inp = H.to_device(H.make_inputs("dcn", cfg, B, seed=3), "cuda")
    label = (torch.rand(B, generator=torch.Generator().manual_seed(4)) < 0.3).float().cuda()
    crit = torch.nn.BCEWithLogitsLoss()
    oa = rankops.Adam(a.parameters(), lr=1e-3, capturable=True)
    ob = rankops.Adam(b.parameters(), lr=1e-3, capturable=True)
    torch.manual_seed(0)
    H.call_model(a, "dcn", inp)  # frozen cross draw
    torch.manual_seed(0)
    H.call_model(b, "dcn", inp)

    def step(model, opt):
        opt.zero_grad(set_to_none=True)
        prob, logit = H.call_model(model, "dcn", inp)
        loss = crit(logit.squeeze(), label)
        loss.backward()
        opt.step()
        return loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step(a, oa)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    oa.zero_grad(set_to_none=True)
    with torch.cuda.graph(graph):
        static_loss = step(a, oa)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    for _ in range(2 + 3):  # warmups + replays (capturing records the step, it does not run it)
        eager_loss = step(b, ob)
    torch.cuda.synchronize()
    assert abs(float(static_loss.detach()) - float(eager_loss.detach())) < 1e-5
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa.detach(), pb.detach(), rtol=1e-5, atol=1e-6, msg=n)


def _dc_step_check(cfg, B, seed, steps):
    model = H.build("deepcrossing", cfg).cuda().train()
    inp = H.make_inputs("deepcrossing", cfg, B, seed=seed)
    label = (torch.rand(B, generator=torch.Generator().manual_seed(seed)) < 0.3).float()
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    names = [n for n, _ in model.named_parameters()]
    opt = rankops.Adam(model.parameters(), lr=1e-3)
    ref_opt = torch.optim.Adam([p[n] for n in names], lr=1e-3)
    crit = torch.nn.BCEWithLogitsLoss()
    dinp = H.to_device(inp, "cuda")
    for step in range(steps):
        opt.zero_grad()
        ref_opt.zero_grad()
        torch.manual_seed(4321 + step)  # per-call residual-unit draws on both sides
        prob, logit = H.call_model(model, "deepcrossing", dinp)
        loss = crit(logit.squeeze(), label.cuda())
        loss.backward()
        torch.manual_seed(4321 + step)
        rprob, rlogit = ref.deepcrossing_forward(p, inp["dense"], inp["category"], cfg.get("internal", 128),
                                                 cfg.get("units", 1))
        rloss = crit(rlogit.squeeze(), label)
        rloss.backward()
        torch.testing.assert_close(logit.detach().cpu(), rlogit.detach(), rtol=1e-4, atol=1e-4)
        for n, prm in model.named_parameters():
            want = p[n].grad
            scale = max(1e-3, float(want.abs().max()))
            torch.testing.assert_close(prm.grad.cpu(), want, rtol=0, atol=2e-4 * scale, msg=f"grad {n} step {step}")
        opt.step()
        ref_opt.step()
        for n, prm in model.named_parameters():
            torch.testing.assert_close(prm.detach().cpu(), p[n].detach(), rtol=1e-4, atol=1e-5,
                                       msg=f"param {n} after step {step}")


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{}, {"units": 3, "internal": 64}, {"units": 0}, {"units": 2, "internal": 600}],
                         ids=["default", "units3", "units0", "wide_internal"])
def test_deepcrossing_train_steps_match_autograd(cfg):
    _dc_step_check(cfg, 1024, seed=2200, steps=3)


def _deepfm_masks(model, B):
    """The dropout multipliers the last train forward drew (rk_dropout_mask on its stream)."""
    from rankops import train as rt
    units = rt.deep_units(model.deep_layers)
    slot = model._dropout.counter - 1
    return [ops.dropout_mask(model._dropout.seed + u, slot, B, lin.out_features, p).cpu() if p > 0 else None
            for u, (lin, bn, relu, p) in enumerate(units)]


def _deepfm_step_check(cfg, B, seed, steps):
    model = H.build("deepfm", cfg).cuda().train()
    fields = list(cfg.get("fields", {f: 0 for f in rankops.deepfm.WECHAT_FIELDS}).keys())
    hidden = len(cfg.get("hidden", [512, 256, 128]))
    inp = H.make_inputs("deepfm", cfg, B, seed=seed)
    label = (torch.rand(B, generator=torch.Generator().manual_seed(seed)) < 0.3).float()
    sd = model.state_dict()
    params = dict(model.named_parameters())
    p = {k: (v.detach().cpu().clone().requires_grad_(True) if k in params else v.detach().cpu().clone())
         for k, v in sd.items()}
    names = list(params)
    opt = rankops.Adam(model.parameters(), lr=1e-3)
    ref_opt = torch.optim.Adam([p[n] for n in names], lr=1e-3)
    crit = torch.nn.BCELoss()
    dinp = H.to_device(inp, "cuda")
    layers = list(model.deep_layers)
    bn_fed_biases = {f"deep_layers.{i}.bias" for i, m in enumerate(layers[:-1])
                     if isinstance(m, torch.nn.Linear) and isinstance(layers[i + 1], torch.nn.BatchNorm1d)}
    for step in range(steps):
        opt.zero_grad()
        ref_opt.zero_grad()
        out = H.call_model(model, "deepfm", dinp)
        loss = crit(out[0].squeeze(), label.cuda())
        loss.backward()
        masks = _deepfm_masks(model, B)
        ref = ref_forward_train(p, inp["category"], fields, hidden, cfg.get("batch_norm", True),
                                cfg.get("dropout", 0.1), masks)
        rloss = crit(ref[0].squeeze(), label)
        rloss.backward()
        for i, (o, r) in enumerate(zip(out, ref)):
            torch.testing.assert_close(o.detach().cpu(), r.detach(), rtol=1e-4, atol=1e-4, msg=f"output {i}")
        for k, v in model.state_dict().items():
            # running statistics and num_batches_tracked; after the first step the running_mean
            # also carries the noise-driven pre-BN biases (skipped below), so compare it once
            if k not in params and (step == 0 or not k.endswith("running_mean")):
                torch.testing.assert_close(v.cpu(), p[k], rtol=1e-4, atol=1e-5, msg=f"buffer {k} step {step}")
        for n, prm in model.named_parameters():
            want = p[n].grad
            scale = max(1e-3, float(want.abs().max()))
            torch.testing.assert_close(prm.grad.cpu(), want, rtol=0, atol=5e-4 * scale, msg=f"grad {n} step {step}")
        opt.step()
        ref_opt.step()
        for n, prm in model.named_parameters():
            if n in bn_fed_biases:
                # a Linear bias right before BatchNorm has a zero true gradient (BN removes any shift);
                # both sides hold rounding noise there, which Adam normalises to +-lr steps
                continue
            _assert_adam_params_close(prm.detach().cpu(), p[n].detach(), lr=1e-3, steps=1,
                                      what=f"param {n} after step {step}")
        # re-synchronise the oracle to the engine so every step is checked from the same state
        # (Adam's noise-level sign flips would otherwise compound across steps)
        with torch.no_grad():
            for k, v in model.state_dict().items():
                p[k].copy_(v.cpu())
            for n, prm in model.named_parameters():
                for key in ("exp_avg", "exp_avg_sq"):
                    ref_opt.state[p[n]][key].copy_(opt.state[prm][key].cpu())


def _assert_adam_params_close(got, want, lr, steps, what):
    """Adam moves every element by about lr per step whatever its gradient's size, so elements whose
    gradient is at rounding-noise level (|g| << the tensor's scale; fp32 sums in another order) may
    step the other way: allow up to 0.5% of elements within 2 lr per step, the rest within 1e-5."""
    diff = (got - want).abs()
    bad = diff > 1e-5 + 1e-4 * want.abs()
    frac = float(bad.float().mean())
    assert frac <= 0.005, f"{what}: {frac:.4%} of elements differ (max {float(diff.max()):.3g})"
    assert float(diff.max()) <= 2 * lr * steps + 1e-5, f"{what}: max diff {float(diff.max()):.3g}"


def ref_forward_train(p, category, fields, hidden, bn, dropout, masks):
    return ref.deepfm_forward_train(p, category, fields, hidden, bn, dropout, masks)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{}, {"batch_norm": False}, {"vocab": H.WECHAT_VOCAB},
                                 {"dim": 32, "fields": {f"field_{i:02d}": 500 + 37 * i for i in range(30)}}],
                         ids=["default", "no_bn", "wechat", "fields30"])
def test_deepfm_train_steps_match_autograd(cfg):
    _deepfm_step_check(cfg, 1024, seed=2300, steps=3)


def _din_masks(model, B):
    from rankops import train as rt
    slot = model._dropout.counter - 1
    return [ops.dropout_mask(model._dropout.seed + u, slot, B, lin.out_features, p).cpu() if p > 0 else None
            for u, (lin, act, bn, p) in enumerate(rt.din_units(model))]


def _din_step_check(cfg, B, seed, steps):
    """DIN train steps (din.py:339-347: forward, BCELoss(prob) + l2_reg, backward, Adam) against the
    oracle's train-mode DIN.forward differentiated by autograd, with the same frozen att_net
    weights and the dropout masks the engine drew."""
    cfg = dict(cfg, interaction_weights="frozen")
    model = H.build("din", cfg).cuda().train()
    att = [t.cpu() for t in model.att_weights.get(torch.device("cuda", 0))]
    hidden = len(cfg.get("hidden", [512, 256, 128]))
    inp = H.make_inputs("din", cfg, B, seed=seed)
    label = (torch.rand(B, generator=torch.Generator().manual_seed(seed)) < 0.3).float()
    params = dict(model.named_parameters())
    p = {k: (v.detach().cpu().clone().requires_grad_(True) if k in params else v.detach().cpu().clone())
         for k, v in model.state_dict().items()}
    names = list(params)
    opt = rankops.Adam(model.parameters(), lr=1e-3)
    ref_opt = torch.optim.Adam([p[n] for n in names], lr=1e-3)
    crit = torch.nn.BCELoss()
    dinp = H.to_device(inp, "cuda")
    for step in range(steps):
        opt.zero_grad()
        ref_opt.zero_grad()
        out = H.call_model(model, "din", dinp)
        loss = crit(out[0].squeeze(), label.cuda()) + out[2]
        loss.backward()
        masks = _din_masks(model, B)
        r = ref.din_forward_train(p, inp["dense"], inp["category"], inp["sequence"], inp["target"], hidden,
                                  cfg.get("batch_norm", True), 0.1, cfg.get("softmax", False), cfg.get("l2", 0.2),
                                  True, att, masks, activation=cfg.get("activation", "dice"))
        rloss = crit(r[0].squeeze(), label) + r[2]
        rloss.backward()
        for i, (o, w) in enumerate(zip(out, r)):
            if isinstance(w, torch.Tensor):
                torch.testing.assert_close(o.detach().cpu().reshape(w.shape), w.detach(), rtol=1e-4, atol=1e-4,
                                           msg=lambda m: f"output {i} step {step}: {m}")
            else:
                assert o == w
        for k, v in model.state_dict().items():
            if k not in params and (step == 0 or not k.endswith("running_mean")):
                torch.testing.assert_close(v.cpu(), p[k], rtol=1e-4, atol=1e-5, msg=lambda m: f"buffer {k} step {step}: {m}")
        for n, prm in model.named_parameters():
            want = p[n].grad
            if want is None:
                assert prm.grad is None or float(prm.grad.abs().max()) == 0.0, n
                continue
            scale = max(1e-3, float(want.abs().max()))
            # the query / history-key gradients sum T positions of att-MLP cross-feature terms that
            # largely cancel (fp32 noise ~2e-3 of the table's largest gradient at T = 50, H = 32)
            tol = (5e-3 if n.startswith("embeddings.") else 5e-4) * scale
            torch.testing.assert_close(prm.grad.cpu(), want, rtol=0, atol=tol, msg=lambda m: f"grad {n} step {step}: {m}")
        opt.step()
        ref_opt.step()
        for n, prm in model.named_parameters():
            if p[n].grad is not None:
                _assert_adam_params_close(prm.detach().cpu(), p[n].detach(), lr=1e-3, steps=1,
                                          what=f"param {n} after step {step}")
        with torch.no_grad():  # re-synchronise the oracle to the engine (see _deepfm_step_check)
            for k, v in model.state_dict().items():
                p[k].copy_(v.cpu())
            for n, prm in model.named_parameters():
                if prm in opt.state and p[n] in ref_opt.state:
                    for key in ("exp_avg", "exp_avg_sq"):
                        ref_opt.state[p[n]][key].copy_(opt.state[prm][key].cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{"T": 20}, {"T": 20, "softmax": True}, {"T": 12, "batch_norm": False, "l2": 0.0},
                                 {"T": 50, "dim": 32, "vocab": H.WECHAT_VOCAB}, {"T": 70, "min_len": 0},
                                 {"T": 20, "activation": "prelu"},
                                 {"T": 16, "activation": "prelu", "batch_norm": False, "softmax": True}],
                         ids=["default", "softmax", "no_bn_no_l2", "bench_shape", "long_empty", "prelu",
                              "prelu_no_bn_softmax"])
def test_din_train_steps_match_autograd(cfg):
    _din_step_check(cfg, 512, seed=2400, steps=2)


@pytest.mark.gpu
def test_din_train_graph_capture_matches_eager():
    """A whole DIN train step (frozen att_net, capturable Adam) captured in one hipGraph gives the
    same parameters as the eager step."""
    cfg = {"T": 20, "interaction_weights": "frozen"}
    inp = H.to_device(H.make_inputs("din", cfg, 256, seed=31), "cuda")
    label = (torch.rand(256, device="cuda") < 0.3).float()
    crit = torch.nn.BCELoss()
    results = []
    for mode in ("eager", "graph"):
        torch.manual_seed(0)
        model = H.build("din", cfg).cuda().train()
        opt = rankops.Adam(model.parameters(), lr=1e-3, capturable=(mode == "graph"))

        def step():
            opt.zero_grad(set_to_none=False)
            out = H.call_model(model, "din", inp)
            (crit(out[0].squeeze(), label) + out[2]).backward()
            opt.step()

        if mode == "eager":
            for _ in range(3):
                step()
        else:
            step()  # draws the frozen weights, allocates the optimizer state
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            g.replay()
            g.replay()
        torch.cuda.synchronize()
        results.append({n: t.detach().cpu().clone() for n, t in model.named_parameters()})
    for n in results[0]:
        torch.testing.assert_close(results[1][n], results[0][n], rtol=1e-5, atol=1e-6, msg=n)


AFM_CATS = ["userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"]


def _afm_step_check(cfg, B, seed, steps):
    """AFM train steps (afm.py:158-180: forward, BCELoss(prediction), backward, Adam) against the
    oracle's AFM.forward (afm.py:92-119) differentiated by autograd."""
    model = H.build("afm", cfg).cuda().train()
    inp = H.make_inputs("afm", cfg, B, seed=seed)
    label = (torch.rand(B, generator=torch.Generator().manual_seed(seed)) < 0.3).float()
    params = dict(model.named_parameters())
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    opt = rankops.Adam(model.parameters(), lr=1e-3)
    ref_opt = torch.optim.Adam([p[n] for n in params], lr=1e-3)
    crit = torch.nn.BCELoss()
    dinp = H.to_device(inp, "cuda")
    for step in range(steps):
        opt.zero_grad()
        ref_opt.zero_grad()
        out = H.call_model(model, "afm", dinp)
        crit(out[0].squeeze(), label.cuda()).backward()
        r = ref.afm_forward(p, inp["dense_input"], inp["category_input"], AFM_CATS)
        crit(r[0].squeeze(), label).backward()
        for i, (o, w) in enumerate(zip(out, r)):
            torch.testing.assert_close(o.detach().cpu(), w.detach(), rtol=1e-4, atol=1e-4,
                                       msg=lambda m: f"output {i} step {step}: {m}")
        for n, prm in params.items():
            want = p[n].grad
            scale = max(1e-4, float(want.abs().max()))
            torch.testing.assert_close(prm.grad.cpu(), want, rtol=0, atol=5e-4 * scale,
                                       msg=lambda m: f"grad {n} step {step}: {m}")
        opt.step()
        ref_opt.step()
        for n, prm in params.items():
            if n == "attention.2.bias":
                # the softmax over pairs is shift-invariant: this bias has a zero true gradient and
                # both sides hold rounding noise, which Adam normalises to +-lr steps
                continue
            _assert_adam_params_close(prm.detach().cpu(), p[n].detach(), lr=1e-3, steps=1,
                                      what=f"param {n} after step {step}")
        with torch.no_grad():
            for n, prm in params.items():
                p[n].copy_(prm.detach().cpu())
                for key in ("exp_avg", "exp_avg_sq"):
                    ref_opt.state[p[n]][key].copy_(opt.state[prm][key].cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{}, {"dim": 32, "att": 64}, {"vocab": H.WECHAT_VOCAB, "dim": 16, "att": 256}],
                         ids=["default", "dim32_att64", "wechat_att256"])
def test_afm_train_steps_match_autograd(cfg):
    _afm_step_check(cfg, 1024, seed=2500, steps=2)


def _bst_masks(model, B, T):
    from rankops import train as rt
    seed, slot = model._dropout.seed, model._dropout.counter - 1
    units, _ = rt.bst_units(model)
    dnn = [ops.dropout_mask(seed + u, slot, B, un[0].out_features, un[3]).cpu() if un[3] > 0 else None
           for u, un in enumerate(units)]
    blocks = []
    for i, blk in enumerate(model.transformer_blocks):
        ps = (blk.dropout.p, blk.ffn[2].p, blk.dropout.p)
        blocks.append([ops.dropout_mask(rt.bst_dropout_seed(seed, i, k), slot, B * T, model.d_model, ps[k]).cpu()
                       if ps[k] > 0 else None for k in range(3)])
    return blocks, dnn


def _bst_step_check(cfg, B, seed, steps):
    """BST train steps (bst.py:266-289: forward, BCELoss(prob), backward, Adam) against the oracle's
    train-mode BSTModel.forward (blocks and dnn with the engine's dropout masks) differentiated by
    autograd."""
    model = H.build("bst", cfg).cuda().train()
    T = cfg.get("T", 50)
    inp = H.make_inputs("bst", cfg, B, seed=seed)
    label = (torch.rand(B, generator=torch.Generator().manual_seed(seed)) < 0.3).float()
    params = dict(model.named_parameters())
    p = {k: (v.detach().cpu().clone().requires_grad_(True) if k in params else v.detach().cpu().clone())
         for k, v in model.state_dict().items()}
    opt = rankops.Adam(model.parameters(), lr=1e-3)
    ref_opt = torch.optim.Adam([p[n] for n in params], lr=1e-3)
    crit = torch.nn.BCELoss()
    dinp = H.to_device(inp, "cuda")
    hidden = len(cfg.get("hidden", [512, 256, 128]))
    bn_fed = {f"dnn.{i}.bias" for i, m in enumerate(model.dnn)
              if isinstance(m, torch.nn.Linear) and i + 1 < len(model.dnn)
              and isinstance(model.dnn[i + 1], torch.nn.BatchNorm1d)}
    for step in range(steps):
        opt.zero_grad()
        ref_opt.zero_grad()
        out = H.call_model(model, "bst", dinp)
        crit(out[0].squeeze(), label.cuda()).backward()
        bm, dm = _bst_masks(model, B, T)
        r = ref.bst_forward_train(p, inp["dense"], inp["category"], inp["seq_feedid"], inp["seq_length"],
                                  cfg.get("heads", 4), cfg.get("blocks", 1), hidden, cfg.get("batch_norm", True), 0.1,
                                  cfg.get("pooling", "sum"), bm, dm)
        crit(r[0].squeeze(), label).backward()
        for i, (o, w) in enumerate(zip(out, r)):
            torch.testing.assert_close(o.detach().cpu(), w.detach(), rtol=1e-4, atol=1e-4,
                                       msg=lambda m: f"output {i} step {step}: {m}")
        for k, v in model.state_dict().items():
            if k not in params and (step == 0 or not k.endswith("running_mean")):
                torch.testing.assert_close(v.cpu(), p[k], rtol=1e-4, atol=1e-5, msg=lambda m: f"buffer {k}: {m}")
        for n, prm in params.items():
            want = p[n].grad
            if want is None:
                assert prm.grad is None or float(prm.grad.abs().max()) == 0.0, n
                continue
            scale = max(1e-3, float(want.abs().max()))  # floor: null-space parameters hold only noise
            # absolute floor 1e-5: gradients reaching the embeddings through the dnn's train-mode
            # BatchNorm (a difference of batch means) carry fp32 cancellation noise of a few 1e-6
            # on both sides (observed 3.5e-6 once on embeddings.userid at the bench shape)
            torch.testing.assert_close(prm.grad.cpu(), want, rtol=0, atol=max(1e-3 * scale, 1e-5),
                                       msg=lambda m: f"grad {n} step {step}: {m}")
        opt.step()
        ref_opt.step()
        for n, prm in params.items():
            # zero true gradients, rounding noise on both sides (Adam turns it into +-lr steps): a
            # Linear bias feeding BatchNorm; w_k's bias (q.(k + b) shifts every key's score of a
            # query by the same q.b, which the softmax removes); with sum pooling over a fixed T the
            # last block's norm2.bias adds the same T * beta to every sample, which the dnn's first
            # BatchNorm removes — caught generically as a numerically-zero oracle gradient
            if (n in bn_fed or n.endswith("w_k.bias") or p[n].grad is None
                    or float(p[n].grad.abs().max()) < 1e-6):
                continue
            _assert_adam_params_close(prm.detach().cpu(), p[n].detach(), lr=1e-3, steps=1,
                                      what=f"param {n} after step {step}")
        with torch.no_grad():
            for k, v in model.state_dict().items():
                p[k].copy_(v.cpu())
            for n, prm in params.items():
                if prm in opt.state and p[n] in ref_opt.state:
                    for key in ("exp_avg", "exp_avg_sq"):
                        ref_opt.state[p[n]][key].copy_(opt.state[prm][key].cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{"T": 20}, {"T": 20, "dim": 32, "blocks": 2, "pooling": "mean"},
                                 {"T": 64, "dim": 128, "max_len": 64, "vocab": H.WECHAT_VOCAB},
                                 {"T": 50, "dim": 32, "max_len": 50}, {"T": 20, "blocks": 0},
                                 {"T": 20, "blocks": 0, "pooling": "mean"}],
                         ids=["reference", "two_blocks_mean", "bench_shape", "reference_T50", "zero_blocks",
                              "zero_blocks_mean"])
def test_bst_train_steps_match_autograd(cfg):
    _bst_step_check(cfg, 256, seed=2600, steps=2)


@pytest.mark.gpu
def test_dropout_mask_rate_and_freshness():
    counter = torch.zeros(1, dtype=torch.int64, device="cuda")
    slot = torch.empty(1, dtype=torch.int64, device="cuda")
    ops.rng_next(counter, slot)
    m1 = ops.dropout_mask(7, slot, 4096, 512, 0.1)
    ops.rng_next(counter, slot)
    m2 = ops.dropout_mask(7, slot, 4096, 512, 0.1)
    keep1 = (m1 > 0).float().mean().item()
    assert abs(keep1 - 0.9) < 0.005
    assert set(torch.unique(m1).tolist()) == {0.0, float(torch.tensor(1 / 0.9, dtype=torch.float32))}
    assert (m1 != m2).float().mean().item() > 0.1  # a new stream draws a new mask
    assert int(counter) == 2


# ------------------------------------------------------------------ eval after training (cache invalidation)

def _eval_vs_oracle(model, name, cfg, inp, interaction=None, seed=17):
    model.eval()
    p = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    torch.manual_seed(seed)
    with torch.no_grad():
        out = H.as_tuple(H.call_model(model, name, inp))
    torch.manual_seed(seed)
    with torch.no_grad():
        want = H.as_tuple(H.call_oracle(name, cfg, p, H.to_device(inp, "cpu"), interaction))
    for i, (o, r) in enumerate(zip(out, want)):
        if isinstance(r, torch.Tensor):
            torch.testing.assert_close(o.detach().cpu(), r, rtol=1e-4, atol=1e-4, msg=lambda m: f"{name}[{i}] {m}")


@pytest.mark.gpu
@pytest.mark.parametrize("name,cfg", [("din", {"T": 20}), ("deepfm", {}), ("bst", {"T": 12, "dim": 16})])
@pytest.mark.parametrize("opt_kind", ["rankops", "torch"])
def test_eval_train_eval_uses_updated_running_stats(name, cfg, opt_kind):
    """The reference loop (din.py:442-446): evaluate, train an epoch, evaluate again.  The second
    eval must fold the BatchNorm / Dice running statistics the train kernels updated (they are
    written through raw pointers), not the fold cached at the first eval."""
    B = 256
    model = H.build(name, cfg).cuda()
    inp = H.to_device(H.make_inputs(name, cfg, B, seed=41), "cuda")
    _eval_vs_oracle(model, name, cfg, inp)  # caches the eval folds
    model.train()
    opt = rankops.Adam(model.parameters(), lr=1e-2) if opt_kind == "rankops" else \
        torch.optim.Adam(model.parameters(), lr=1e-2)
    label = (torch.rand(B, generator=torch.Generator().manual_seed(3)) < 0.3).float().cuda()
    for _ in range(3):
        opt.zero_grad()
        out = H.as_tuple(H.call_model(model, name, inp))
        logit_loss = name == "bst"
        loss = torch.nn.functional.binary_cross_entropy_with_logits(out[1].squeeze(), label) if logit_loss else \
            torch.nn.functional.binary_cross_entropy(out[0].squeeze(), label)
        loss.backward()
        opt.step()
    stats = [m.running_mean for m in model.modules() if isinstance(m, torch.nn.BatchNorm1d)]
    assert stats, "config has no BatchNorm"
    _eval_vs_oracle(model, name, cfg, inp)


@pytest.mark.gpu
def test_graph_replayed_train_steps_then_eval():
    """Replays of a captured DIN train step change weights and running statistics without any
    tensor-version bump; model.eval() must still invalidate the eval folds and packed weights."""
    cfg = {"T": 20, "interaction_weights": "frozen"}
    B = 256
    inp = H.to_device(H.make_inputs("din", cfg, B, seed=51), "cuda")
    label = (torch.rand(B, generator=torch.Generator().manual_seed(5)) < 0.3).float().cuda()
    torch.manual_seed(0)
    model = H.build("din", cfg).cuda()
    _eval_vs_oracle(model, "din", cfg, inp)  # draws the frozen att_net (same seed on both sides)
    att = [t.detach().cpu() for t in model.att_weights._cached[1]]
    _eval_vs_oracle(model, "din", cfg, inp, interaction=att)
    model.train()
    opt = rankops.Adam(model.parameters(), lr=1e-2, capturable=True)

    def step():
        opt.zero_grad(set_to_none=False)
        out = H.call_model(model, "din", inp)
        (torch.nn.functional.binary_cross_entropy(out[0].squeeze(), label) + out[2]).backward()
        opt.step()

    step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(4):
        g.replay()
    torch.cuda.synchronize()
    _eval_vs_oracle(model, "din", cfg, inp, interaction=att)


def _attn_reference(qkv, B, T, d, heads, seq_len, dctx):
    """bst.py:72-83 in float64 autograd: softmax(mask(Q K^T / sqrt(dh))) V, mask = positions >= len."""
    dh = d // heads
    x = qkv.detach().double().requires_grad_(True)
    q, k, v = (x[:, i * d:(i + 1) * d].view(B, T, heads, dh).transpose(1, 2) for i in range(3))
    s = torch.matmul(q, k.transpose(-2, -1)) / np.sqrt(dh)
    mask = torch.arange(T)[None, :] >= seq_len.cpu()[:, None]
    s = s.masked_fill(mask[:, None, None, :], float("-inf"))
    p = torch.softmax(s, dim=-1)
    ctx = torch.matmul(p, v).transpose(1, 2).reshape(B * T, d)
    ctx.backward(dctx.double())
    return p, ctx, x.grad


@pytest.mark.gpu
@pytest.mark.parametrize("T,d,heads", [(64, 128, 4), (50, 32, 4), (20, 32, 4), (1, 16, 2), (17, 48, 1), (33, 256, 4),
                                       (64, 256, 4), (7, 12, 3)])
def test_bst_attention_train_kernels_match_autograd(T, d, heads):
    """rk_bst_attn_train_forward / _backward (MFMA, T and dh zero-padded to 16) against float64 autograd
    over every padding case: T < 16, T = 16k + 1, dh = 4, 12, 16, 48, 64; lengths 1..T (length 0 gives
    NaN rows in the reference and here, checked separately)."""
    g = torch.Generator().manual_seed(T * 1000 + d)
    B = 37
    qkv = torch.randn(B * T, 3 * d, generator=g)
    dctx = torch.randn(B * T, d, generator=g)
    seq_len = torch.randint(1, T + 1, (B,), generator=g)
    seq_len[0], seq_len[-1] = 1, T
    p_ref, c_ref, dx_ref = _attn_reference(qkv, B, T, d, heads, seq_len, dctx)
    dev = torch.device("cuda")
    qkv_d, dctx_d, len_d = qkv.to(dev), dctx.to(dev), seq_len.to(dev)
    probs = torch.full((B, heads, T, T), float("nan"), device=dev)
    ctx = torch.full((B * T, d), float("nan"), device=dev)
    dqkv = torch.full((B * T, 3 * d), float("nan"), device=dev)
    ops.bst_attn_train_forward(qkv_d, B, T, d, heads, len_d, probs, ctx)
    ops.bst_attn_train_backward(qkv_d, probs, dctx_d, B, T, d, heads, dqkv)
    torch.cuda.synchronize()
    torch.testing.assert_close(probs.cpu().double(), p_ref.detach(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(ctx.cpu().double(), c_ref.detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(dqkv.cpu().double(), dx_ref, atol=1e-4, rtol=1e-4)
    if T % 4 == 0 and (d // heads) % 4 == 0:
        # no P output (probs = NULL): the same context, bit for bit
        ctx2 = torch.full((B * T, d), float("nan"), device=dev)
        ops.bst_attn_train_forward(qkv_d, B, T, d, heads, len_d, None, ctx2)
        torch.cuda.synchronize()
        assert torch.equal(ctx2, ctx)


@pytest.mark.gpu
def test_bst_attention_train_length_zero_is_nan():
    """A sample with no valid key: the reference's softmax over an all -inf row is NaN (bst.py:80-82)."""
    B, T, d, heads = 3, 20, 32, 4
    qkv = torch.randn(B * T, 3 * d, device="cuda")
    seq_len = torch.tensor([5, 0, 20], device="cuda")
    probs = torch.empty(B, heads, T, T, device="cuda")
    ctx = torch.empty(B * T, d, device="cuda")
    ops.bst_attn_train_forward(qkv, B, T, d, heads, seq_len, probs, ctx)
    torch.cuda.synchronize()
    assert torch.isnan(probs[1]).all() and torch.isnan(ctx[T:2 * T]).all()
    assert torch.isfinite(probs[0]).all() and torch.isfinite(ctx[:T]).all() and torch.isfinite(ctx[2 * T:]).all()


# Tall-skinny shapes (gemm_rows.hip: M >= 32 x 4 x CUs rows, reduction <= 128) — the BST / DIN training
# GEMMs.  M is deliberately not a multiple of 32.
ROWS_M = 131072 + 77


@pytest.mark.gpu
@pytest.mark.parametrize("TB", [0, 1])
@pytest.mark.parametrize("N,R", [(128, 128), (64, 128), (200, 36), (7, 12), (384, 64), (32, 100)])
@pytest.mark.parametrize("masked", [False, True])
def test_gemm_rows_tall_skinny_matches_fp64(TB, N, R, masked):
    M = ROWS_M
    A, B, mask, want, _ = _gemm_case(0, TB, M, N, R, masked, seed=N * 13 + R + TB)
    C = torch.full((M, N), 7.0, device="cuda")
    Ad, Bd = A.cuda(), B.cuda()
    md = mask.cuda() if mask is not None else None
    ops.gemm(0, TB, M, N, R, Ad, Ad.stride(0), Bd, Bd.stride(0), C, A_mask=md)
    tol = 1e-4 * max(1.0, float(want.abs().max()))
    torch.testing.assert_close(C.cpu().double(), want, rtol=0, atol=tol)
    ops.gemm(0, TB, M, N, R, Ad, Ad.stride(0), Bd, Bd.stride(0), C, A_mask=md, accumulate=True)
    torch.testing.assert_close(C.cpu().double(), 2 * want, rtol=0, atol=2 * tol)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [32768 + 5, 65536 + 77])
@pytest.mark.parametrize("N,R", [(128, 128), (384, 64), (7, 32)])
def test_gemm_rows_mid_size_matches_fp64(M, N, R):
    """The gemm_rows path from 4 slabs per CU (one or two slabs per resident wave): plain and
    accumulating products against float64."""
    A, B, mask, want, _ = _gemm_case(0, 1, M, N, R, False, seed=M + N)
    C = torch.full((M, N), 7.0, device="cuda")
    Ad, Bd = A.cuda(), B.cuda()
    ops.gemm(0, 1, M, N, R, Ad, Ad.stride(0), Bd, Bd.stride(0), C)
    tol = 1e-4 * max(1.0, float(want.abs().max()))
    torch.testing.assert_close(C.cpu().double(), want, rtol=0, atol=tol)
    ops.gemm(0, 1, M, N, R, Ad, Ad.stride(0), Bd, Bd.stride(0), C, accumulate=True)
    torch.testing.assert_close(C.cpu().double(), 2 * want, rtol=0, atol=2 * tol)


@pytest.mark.gpu
@pytest.mark.parametrize("N,K,act,periodic,residual", [(128, 128, "none", True, False), (128, 128, "relu", False, True),
                                                       (64, 128, "relu", False, False), (32, 64, "none", False, False),
                                                       (200, 40, "leaky", False, False), (5, 8, "none", True, True)])
def test_linear_tall_skinny_matches_fp64(N, K, act, periodic, residual):
    """rk_linear over M = 131149 rows (gemm_rows path): bias, x + periodic addend (BST positions),
    residual, activation, strided output (ldy > N)."""
    M = ROWS_M
    g = torch.Generator().manual_seed(N + K)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    per = torch.randn(64, K, generator=g) if periodic else None
    res = torch.randn(M, N, generator=g) if residual else None
    xin = x.double() + (per.double().repeat(M // 64 + 1, 1)[:M] if periodic else 0)
    want = xin @ w.double().t() + b.double()
    if residual:
        want = res.double() + want
    if act == "relu":
        want = want.clamp_min(0)
    elif act == "leaky":
        want = torch.where(want > 0, want, want * 0.01)
    out = torch.full((M, N + 3), 7.0, device="cuda")
    bd = b.cuda()
    rd = res.cuda() if residual else None
    ep = ops.make_epilogue(bias=bd, act=act if act != "none" else None, slope=0.01, residual=rd,
                           ld_residual=N if residual else 0)
    ops.linear(x.cuda(), w.cuda(), None, y_ptr=out.data_ptr(), ldy=N + 3,
               x_periodic=per.cuda() if periodic else None, x_period=64 if periodic else 0, epilogue=ep)
    torch.cuda.synchronize()
    torch.testing.assert_close(out[:, :N].cpu().double(), want, rtol=1e-4, atol=1e-4)
    assert float((out[:, N:] - 7.0).abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("M,N", [(128, 128), (64, 128), (200, 36), (7, 12), (256, 512)])
@pytest.mark.parametrize("masked", [False, True])
def test_gemm_cols_weight_gradient_matches_fp64(M, N, masked):
    """rk_gemm(trans_a, trans_b) over R = 131149 rows (the weight-gradient shape: split reduction + atomics):
    C = opA^T-reduction and the bias row sums, fresh and accumulated."""
    R = ROWS_M
    A, B, mask, want, rs = _gemm_case(1, 1, M, N, R, masked, seed=M + 3 * N)
    C = torch.full((M, N), 7.0, device="cuda")
    sums = torch.full((M,), 7.0, device="cuda")
    Ad, Bd = A.cuda(), B.cuda()
    md = mask.cuda() if mask is not None else None
    ops.gemm(1, 1, M, N, R, Ad, Ad.stride(0), Bd, Bd.stride(0), C, A_mask=md, row_sums=sums)
    tol = 2e-4 * max(1.0, float(want.abs().max()))
    torch.testing.assert_close(C.cpu().double(), want, rtol=0, atol=tol)
    torch.testing.assert_close(sums.cpu().double(), rs, rtol=0, atol=tol)
    ops.gemm(1, 1, M, N, R, Ad, Ad.stride(0), Bd, Bd.stride(0), C, A_mask=md, row_sums=sums, accumulate=True)
    torch.testing.assert_close(C.cpu().double(), 2 * want, rtol=0, atol=2 * tol)
    torch.testing.assert_close(sums.cpu().double(), 2 * rs, rtol=0, atol=2 * tol)


@pytest.mark.gpu
@pytest.mark.parametrize("N,K,R,col", [(128, 128, 70001, 128), (256, 128, 4099, 0), (132, 260, 65, 4), (8, 4, 1, 0)])
def test_gemm_wgrad_strided_views_match_fp64(N, K, R, col):
    """rk_gemm_wgrad (ops.gemm with both operands transposed) on column views of a wider matrix
    (dK = dqkv[:, d:2d] as in the BST backward): row pitch lda > N, ragged R, N/K off the 128 tile."""
    g = torch.Generator().manual_seed(N + K + R)
    wide = torch.randn(R, col + N + 8, generator=g)
    X = torch.randn(R, K, generator=g)
    A = wide[:, col:col + N]
    want = A.double().t() @ X.double()
    rs = A.double().sum(0)
    wd, Xd = wide.cuda(), X.cuda()
    Ad = wd[:, col:col + N]
    C = torch.full((N, K), 7.0, device="cuda")
    sums = torch.full((N,), 7.0, device="cuda")
    ops.gemm(1, 1, N, K, R, Ad, wd.stride(0), Xd, Xd.stride(0), C, row_sums=sums)
    tol = 2e-4 * max(1.0, float(want.abs().max()))
    torch.testing.assert_close(C.cpu().double(), want, rtol=0, atol=tol)
    torch.testing.assert_close(sums.cpu().double(), rs, rtol=0, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("B,T,d", [(37, 64, 128), (5, 9, 6), (130, 50, 32)])
def test_embedding_backward_seq_matches_index_add(B, T, d):
    """rk_embedding_backward_seq (BST's sequence gradient without the sort): runs of equal
    consecutive ids inside a sample, padded tails of one id shared by neighbouring samples, and a
    whole sample of one id, against torch.index_add_ in float64."""
    g = torch.Generator().manual_seed(B * T + d)
    V = 40
    seq = torch.randint(0, V, (B, T), generator=g)
    for b in range(B):
        n = int(torch.randint(1, T + 1, (1,), generator=g))
        seq[b, n:] = 0  # padded tail
        if b % 3 == 1 and T > 4:
            seq[b, 1:4] = seq[b, 1]  # a run in the middle
    seq[0, :] = 7  # one id for the whole sample
    dx = torch.randn(B * T, d, generator=g)
    want = torch.zeros(V, d, dtype=torch.float64).index_add_(0, seq.reshape(-1), dx.double())
    grad = torch.zeros(V, d, device="cuda")
    assert ops.embedding_backward_seq(grad, seq.cuda(), dx.cuda())
    torch.testing.assert_close(grad.cpu().double(), want, rtol=0, atol=1e-4 * max(1.0, float(want.abs().max())))


@pytest.mark.gpu
def test_embedding_backward_seq_out_of_range_ids():
    """an out-of-range id (-2 included) is skipped and flagged; the gradients of the
    valid positions around it are still applied."""
    import rankops
    rankops.error_flags()
    V, d = 10, 8
    seq = torch.tensor([[5, -2, 7, 7], [3, 3, V + 4, 3], [-2, -2, 1, 0]])
    dx = torch.randn(seq.numel(), d, generator=torch.Generator().manual_seed(3))
    ok = (seq >= 0) & (seq < V)
    want = torch.zeros(V, d, dtype=torch.float64).index_add_(0, seq.reshape(-1)[ok.reshape(-1)],
                                                              dx[ok.reshape(-1)].double())
    grad = torch.zeros(V, d, device="cuda")
    assert ops.embedding_backward_seq(grad, seq.cuda(), dx.cuda())
    torch.testing.assert_close(grad.cpu().double(), want, rtol=0, atol=1e-5)
    assert rankops.error_flags() == rankops._lib.RK_FLAG_INDEX_OOB


@pytest.mark.gpu
def test_pool_ln_backward_misaligned_workspace_is_unsupported():
    """a workspace pointer that is not 16-B aligned is refused (RK_ERR_UNSUPPORTED)
    instead of reaching the scalar kernel, which has no pooled-row form."""
    lib = rankops_lib()
    B, T, d = 4, 8, 32
    r = torch.randn(B * T, d, device="cuda")
    mean = torch.zeros(B * T, device="cuda")
    rstd = torch.ones(B * T, device="cuda")
    gamma = torch.ones(d, device="cuda")
    drow = torch.randn(B, 16 + d, device="cuda")
    dr, d_o = torch.empty_like(r), torch.empty_like(r)
    dg, db = torch.empty(d, device="cuda"), torch.empty(d, device="cuda")
    nws = lib.rk_bst_ln_backward_workspace_floats(d)
    ws = torch.empty(nws + 4, device="cuda")
    seq_len = torch.full((B,), T, dtype=torch.int64, device="cuda")
    P = ops.ptr
    args = lambda w: (P(drow), drow.stride(0), 16, T, P(seq_len), 0, P(r), P(mean), P(rstd), P(gamma), B * T, d,  # noqa
                      0.0, 0, None, P(dr), P(d_o), P(dg), P(db), w, nws, None)
    assert lib.rk_bst_pool_ln_backward(*args(ws.data_ptr() + 4)) == 4  # RK_ERR_UNSUPPORTED
    assert lib.rk_bst_pool_ln_backward(*args(ws.data_ptr())) == 0
    torch.cuda.synchronize()


def rankops_lib():
    import rankops
    return rankops.load_library()


@pytest.mark.gpu
def test_adam_fast_step_matches_torch_over_storage_changes():
    """rankops.Adam's cached eager step (same gradient storages every step) against torch.optim.Adam,
    through gradient storages that change, a skipped parameter, an lr change and a state_dict
    round trip."""
    g = torch.Generator().manual_seed(21)
    shapes = [(300, 16), (7,), (4096,)]
    pa = [torch.nn.Parameter(torch.randn(s, generator=g).cuda()) for s in shapes]
    qa = [torch.nn.Parameter(p.detach().clone()) for p in pa]
    ours = rankops.Adam(pa, lr=1e-3)
    theirs = torch.optim.Adam(qa, lr=1e-3)
    bufs = [torch.empty(s, device="cuda") for s in shapes]  # the same gradient storages each step
    for step in range(12):
        for a, b, buf in zip(pa, qa, bufs):
            gr = torch.randn(a.shape, generator=g).cuda()
            if step in (5, 6):  # new storages for two steps
                a.grad = gr.clone()
            else:
                buf.copy_(gr)
                a.grad = buf
            b.grad = gr.clone()
        if step == 8:
            pa[1].grad = None
            qa[1].grad = None
        if step == 10:
            for grp in (ours.param_groups[0], theirs.param_groups[0]):
                grp["lr"] = 5e-4
        ours.step()
        theirs.step()
        for a, b in zip(pa, qa):
            torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-6, atol=1e-6, msg=lambda m: f"step {step}: {m}")
    assert [float(ours.state[p]["step"]) for p in pa] == [12.0, 11.0, 12.0]
    # (a deep copy: Optimizer.load_state_dict keeps same-device tensors as they are, so the two
    # optimizers would otherwise share their moment buffers)
    import copy
    ours.load_state_dict(copy.deepcopy(theirs.state_dict()))
    for a, b, buf in zip(pa, qa, bufs):
        buf.copy_(torch.ones_like(buf))
        a.grad, b.grad = buf, buf.clone()
    ours.step()
    theirs.step()
    for a, b in zip(pa, qa):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,p", [(131072 + 37, 128, 0.1), (4096, 64, 0.0), (333, 32, 0.25)])
def test_linear_res_dropout_ln_matches_two_launch_path(M, K, p):
    """rk_linear_res_dropout_ln (the BST O / FFN2 projection with the residual LayerNorm in its
    epilogue) against rk_linear + rk_bst_res_dropout_ln_forward on the same inputs and dropout
    stream: the same projection and mask (r bit-identical), LayerNorm statistics summed in another
    order (1e-5)."""
    g = torch.Generator().manual_seed(M + K)
    d = 128
    x = torch.randn(M, K, generator=g).cuda()
    w = (0.1 * torch.randn(d, K, generator=g)).cuda()
    b = torch.randn(d, generator=g).cuda()
    base = torch.randn(M, d, generator=g).cuda()
    ln = torch.nn.LayerNorm(d).cuda()
    with torch.no_grad():
        ln.weight.copy_(1 + 0.1 * torch.randn(d, generator=g))
        ln.bias.copy_(0.1 * torch.randn(d, generator=g))
    slot = torch.full((1,), 5, dtype=torch.int64, device="cuda")
    outs = []
    for fused in (True, False):
        r, y = torch.empty(M, d, device="cuda"), torch.empty(M, d, device="cuda")
        mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
        if fused:
            assert ops.linear_res_dropout_ln(x, w, b, base, p, 1234, slot, ln, r, y, mean, rstd)
        else:
            o = torch.empty(M, d, device="cuda")
            ops.linear(x, w, o, epilogue=ops.make_epilogue(bias=b))
            ops.bst_res_dropout_ln_forward(base, o, p, 1234, slot, ln, r, y, mean, rstd)
        torch.cuda.synchronize()
        outs.append((r, y, mean, rstd))
    (r1, y1, m1, s1), (r2, y2, m2, s2) = outs
    if M >= 32768:  # both projections on gemm_rows: the same products, the same mask
        assert torch.equal(r1, r2)
    else:  # rk_linear takes its generic kernel at this M (another k order)
        torch.testing.assert_close(r1, r2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(m1, m2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(s1, s2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(y1, y2, rtol=1e-5, atol=1e-5)
    # and against float64 torch on the fused path's own r
    rr = r1.double()
    want = torch.nn.functional.layer_norm(rr, (d,), ln.weight.double(), ln.bias.double(), ln.eps)
    torch.testing.assert_close(y1.double(), want, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_adam_fast_step_cache_hits_with_set_to_none_and_frees_old_grads():
    """the cached eager step must not keep the previous step's gradients alive.  With the
    reference's loop body (zero_grad(set_to_none=True), forward, backward, step) the old gradient
    storages are freed, the caching allocator hands the same addresses back, and the argument block
    is reused instead of rebuilt every step."""
    import weakref
    torch.manual_seed(0)
    model = H.build("dcn", {"interaction_weights": "frozen"}).cuda().train()
    inp = H.to_device(H.make_inputs("dcn", {}, 256, seed=3), "cuda")
    label = (torch.rand(256, device="cuda") < 0.3).float()
    opt = rankops.Adam(model.parameters(), lr=1e-3)
    crit = torch.nn.BCEWithLogitsLoss()
    old = []
    for step in range(6):
        opt.zero_grad(set_to_none=True)
        out = H.as_tuple(H.call_model(model, "dcn", inp))
        crit(out[1].squeeze(), label).backward()
        old.append([weakref.ref(p.grad) for p in model.parameters() if p.grad is not None])
        opt.step()
    opt.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    assert all(r() is None for refs in old for r in refs)  # no step's gradient is held by the cache
    assert getattr(opt, "_fast_builds", 0) <= 2  # built on the first fast step, then reused
