"""DIN (Deep Interest Network) on the rankops engine — drop-in for algorithm/DIN/din.py.

`DIN(vocab_dir, hidden_units=None, activation='dice', dropout_rate=0.1, batch_norm=True,
use_softmax=False, l2_lambda=0.2, mini_batch_aware_regularization=True)` keeps the reference
constructor, creation order, state_dict keys (`embeddings.*`, `fcn.N.*` incl. Dice's
`alpha`/`bn.running_*`, `output_layer.*`; din.py:225-285) and
`forward(dense, category, sequence, target) -> (probability, logit, l2_reg)` (din.py:294-323).

`embedding_dim` (keyword, default 16 = the reference) widens the target/history embeddings
for the benchmark configuration (H = 32).

Launches: rk_concat_gather builds [dense | category | target] in one row buffer, the
rk_din_attention kernel (din.py:42-84) writes the attention output straight into the same
row, rk_row_l2norm_mean gives the l2 term (din.py:318-322), and the fcn stack runs on
rk_linear with Dice + BatchNorm in the epilogue and the output layer + sigmoid fused last.
The attention MLP is drawn per call like the reference (din.py:61-67) or frozen.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import common, ops, train
from .common import PACKED, fused_mlp_fits
from .common import EngineModule, InteractionWeights, Layer, check_eval, din_attention_spec, draw_din_attention, \
    load_vocabulary, run_tail, \
    table_rows

FIELDS = ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list")
SEQ_KEY = "his_read_comment_7d_seq"


class _DiceTrain(torch.autograd.Function):
    """Dice with batch statistics (BatchNorm1d in train mode, running statistics updated):
    rk_dice_train_forward / rk_dice_backward."""

    @staticmethod
    def forward(ctx, x, alpha, dice):
        n = x.shape[1]
        f32 = dict(device=x.device, dtype=torch.float32)
        y = torch.empty_like(x)
        mean, invstd = torch.empty(n, **f32), torch.empty(n, **f32)
        ops.dice_train_forward(x, None, dice, y, mean, invstd, torch.empty(2 * n, device=x.device,
                                                                          dtype=torch.float64))
        ctx.save_for_backward(x, mean, invstd)
        ctx.dice = dice
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, invstd = ctx.saved_tensors
        dy = dy.contiguous()
        n = x.shape[1]
        dx = torch.empty_like(x)
        dalpha = torch.empty(n, device=x.device, dtype=torch.float32)
        ops.dice_backward(dy, x, None, ctx.dice, mean, invstd, torch.empty(3 * n, device=x.device,
                                                                          dtype=torch.float64), dx, dalpha)
        return dx, dalpha, None


class Dice(nn.Module):
    """Dice activation (din.py:26-36): alpha * (1 - p) * x + p * x, p = sigmoid(BatchNorm1d(x))
    with an affine-free BatchNorm (its eps 1e-5; the module's own eps is unused, as in the
    reference).  Same parameters/buffers as the reference.  Inside DIN it runs fused in the fcn
    epilogue; called on its own, eval uses rk_dice_forward (running statistics folded by
    rk_bn_fold) and train mode rk_dice_train_forward / rk_dice_backward (batch statistics)."""

    def __init__(self, num_features, eps=1e-9):
        super().__init__()
        self.eps = eps
        self.alpha = nn.Parameter(torch.zeros(num_features))
        self.bn = nn.BatchNorm1d(num_features, affine=False)
        self._fold = common.FoldedBN()

    def forward(self, x):
        x = ops.as_f32(x, "Dice input")
        if x.dim() != 2 or x.shape[1] != self.alpha.numel():
            raise ValueError(f"rankops Dice: expected [batch, {self.alpha.numel()}], got {tuple(x.shape)}")
        x = x.contiguous()
        if self.bn.training or not self.bn.track_running_stats or self.bn.running_mean is None:
            if self.bn.momentum is None:
                raise NotImplementedError("rankops Dice: BatchNorm momentum=None (cumulative average)")
            if x.shape[0] < 2:
                raise ValueError("Expected more than 1 value per channel when training (BatchNorm1d)")
            return _DiceTrain.apply(x, self.alpha, self)
        scale, shift = self._fold(self.bn)
        y = torch.empty_like(x)
        ops.dice_forward(x, scale, shift, self.alpha, y)
        return y


def din_attention(query, keys, keys_length, is_softmax=False, *, weights=None):
    """din_attention(query[B,H], keys[B,T,H], keys_length[B], is_softmax=False) -> [B,H]
    (din.py:42-84) on rk_din_attention_dense.  The attention MLP Linear(4H,64), Linear(64,32),
    Linear(32,1) is drawn from the CPU generator on every call like the reference (din.py:61-67);
    `weights` = (W1, b1, W2, b2, W3, b3) device tensors replaces the draw."""
    query = ops.as_f32(query, "query")
    keys = ops.as_f32(keys, "keys")
    keys_length = ops.as_index(keys_length, "keys_length")
    if keys.dim() != 3 or query.dim() != 2 or query.shape[0] != keys.shape[0] or query.shape[1] != keys.shape[2]:
        raise ValueError(f"din_attention: query {tuple(query.shape)} and keys {tuple(keys.shape)} do not match")
    B, T, H = keys.shape
    if keys.stride(2) != 1 or keys.stride(1) % 4 or keys.stride(0) % 4 or keys.data_ptr() % 16:
        keys = keys.contiguous()
    if query.stride(1) != 1:
        query = query.contiguous()
    if weights is None:
        weights = [t.to(keys.device) for t in draw_din_attention(H)]
    out = torch.empty(B, H, device=keys.device, dtype=torch.float32)
    if B == 0:
        return out
    ops.din_attention_dense(query, keys, keys_length.contiguous(), weights, is_softmax, out)
    return out


def din_attention_gather(query, keys_table, seq, keys_length, is_softmax=False, weights=None):
    """din_attention with the history given as (embedding table, index [B,T]) — the gather
    din.py:300-303 does before the call happens inside the kernel (rk_din_attention).
    `weights` as for din_attention."""
    query = ops.as_f32(query, "query")
    seq = ops.as_index(seq, "keys index")
    keys_length = ops.as_index(keys_length, "keys_length")
    B, H = query.shape
    T = seq.shape[1]
    if weights is None:
        weights = [t.to(query.device) for t in draw_din_attention(H)]
    out = torch.empty(B, H, device=query.device, dtype=torch.float32)
    ops.din_attention(query.data_ptr(), query.stride(0), keys_table, seq.contiguous(), keys_length, T, H, weights,
                      is_softmax, out.data_ptr(), out.stride(0), B, query.device)
    return out


class DIN(EngineModule):
    def __init__(self, vocab_dir, hidden_units=None, activation='dice', dropout_rate=0.1, batch_norm=True,
                 use_softmax=False, l2_lambda=0.2, mini_batch_aware_regularization=True, *, vocab_sizes=None,
                 embedding_dim=16, interaction_weights="per_call"):
        super().__init__()
        if hidden_units is None:
            hidden_units = [512, 256, 128]
        self.activation = activation
        self.dropout_rate = dropout_rate
        self.batch_norm = batch_norm
        self.use_softmax = use_softmax
        self.l2_lambda = l2_lambda
        self.mini_batch_aware_regularization = mini_batch_aware_regularization
        self.vocab_sizes = {f: table_rows(vocab_dir, f, vocab_sizes) for f in FIELDS}
        self.num_dense_features = 16
        self.embeddings = nn.ModuleDict({
            "userid": nn.Embedding(self.vocab_sizes["userid"], 16),
            "device": nn.Embedding(self.vocab_sizes["device"], 2),
            "authorid": nn.Embedding(self.vocab_sizes["authorid"], 4),
            "bgm_song_id": nn.Embedding(self.vocab_sizes["bgm_song_id"], 4),
            "bgm_singer_id": nn.Embedding(self.vocab_sizes["bgm_singer_id"], 4),
            "manual_tag_list": nn.Embedding(self.vocab_sizes["manual_tag_list"], 4),
            "feedid": nn.Embedding(self.vocab_sizes["feedid"], embedding_dim),
            SEQ_KEY: nn.Embedding(self.vocab_sizes["feedid"], embedding_dim),
        })
        width = self.num_dense_features
        for key in ("userid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"):
            width += self.embeddings[key].embedding_dim
        width += self.embeddings["feedid"].embedding_dim + self.embeddings[SEQ_KEY].embedding_dim
        self.fcn = nn.ModuleList()
        self._tail = []
        for unit in hidden_units:
            lin = nn.Linear(width, unit)
            self.fcn.append(lin)
            if activation == 'dice':
                act = Dice(unit)
                kind = "dice"
            else:
                act = nn.PReLU()
                kind = "prelu"
            self.fcn.append(act)
            bn = None
            if batch_norm:
                bn = nn.BatchNorm1d(unit)
                self.fcn.append(bn)
            if dropout_rate > 0:
                self.fcn.append(nn.Dropout(dropout_rate))
            self._tail.append(Layer(lin, act=kind, act_module=act, post_bn=bn))
            width = unit
        self.output_layer = nn.Linear(width, 1)
        self.att_weights = InteractionWeights(
            interaction_weights, lambda: din_attention_spec(self.embeddings[SEQ_KEY].embedding_dim))
        self._dropout = train.DropoutStreams()

    def _load_vocabulary(self, vocab_dir, filename):
        return load_vocabulary(vocab_dir, filename)

    def _plan(self, dense, category, sequence, target):
        """Row layout [dense | category | target | attention] and the gather segments (din.py:296-310)."""
        dense_cols = [ops.as_f32(v, f"dense[{k!r}]") for k, v in dense.items()]
        B = dense_cols[0].shape[0]
        dev = dense_cols[0].device
        segs = [ops.dense_segment(v, 1, i) for i, v in enumerate(dense_cols)]
        col = len(dense_cols)
        cat_col0 = col
        lookups = []  # (table weight, index, column) for the training backward
        for name, emb in self.embeddings.items():
            if name in category:
                idx = ops.as_index(category[name], f"category[{name!r}]")
                segs.append(ops.table_segment(emb.weight, idx, col))
                lookups.append((emb.weight, idx, col))
                col += emb.embedding_dim
        tgt_emb = self.embeddings["feedid"]
        H = tgt_emb.embedding_dim
        tgt_idx = ops.as_index(target["feedid"], "target['feedid']")
        segs.append(ops.table_segment(tgt_emb.weight, tgt_idx, col))
        lookups.append((tgt_emb.weight, tgt_idx, col))
        q_col = col
        att_col = q_col + H
        width = att_col + self.embeddings[SEQ_KEY].embedding_dim
        seq = ops.as_index(sequence[SEQ_KEY], f"sequence[{SEQ_KEY!r}]").contiguous()
        seq_len = ops.as_index(sequence[f"{SEQ_KEY}_length"], "sequence length")
        fused = (common.FUSED_DIN and H in (8, 16, 32) and width <= 255 and len(segs) <= 32
                 and self.embeddings[SEQ_KEY].embedding_dim == H
                 and fused_mlp_fits(width, [l.linear.out_features for l in self._tail])
                 and (width, seq.shape[1], H) not in self.__dict__.get("_unfusable", ()))
        return dict(B=B, dev=dev, segs=segs, cat_col0=cat_col0, q_col=q_col, att_col=att_col, width=width, H=H,
                    seq=seq, seq_len=seq_len, fused=fused, keep=(dense_cols, category, target), lookups=lookups,
                    seq_key=SEQ_KEY, want_l2=self.mini_batch_aware_regularization and self.l2_lambda > 0)

    def _att_image(self, w, H):
        """The attention weights pre-split into din_forward_kernel's LDS image: cached for frozen
        H2 weights (they live on the device for good), packed per call otherwise."""
        if self.att_weights.mode != "frozen":
            return ops.din_pack_attention(w, H)
        k = common._key(w) + (H,)
        if getattr(self, "_att_img", None) is None or self._att_img[0] != k:
            self._att_img = (k, ops.din_pack_attention(w, H))
        return self._att_img[1]

    def _launch_fused(self, pl, w, logit, prob, l2_reg):
        layers = [ops.make_mlp_layer(l.linear.weight, PACKED(l.linear.weight), **l.epilogue_kwargs())
                  for l in self._tail]
        img = self._att_image(w, pl["H"])
        head = ops.make_epilogue(head_w=self.output_layer.weight, head_b=self.output_layer.bias,
                                 head_logit=logit, head_prob=prob)
        ops.din_forward(pl["segs"], pl["width"], pl["q_col"], pl["att_col"], self.embeddings[SEQ_KEY].weight,
                        pl["seq"], pl["seq_len"], pl["H"], w, self.use_softmax, layers, head, pl["B"], pl["dev"],
                        l2_col0=pl["cat_col0"], l2_scale=float(self.l2_lambda),
                        l2_out=l2_reg if isinstance(l2_reg, torch.Tensor) else None, att_image=img)

    def prepare(self, dense, category, sequence, target):
        """An eval forward bound to these input tensors (the single-kernel analogue of capturing
        the forward in a hipGraph): returns `run()` that recomputes the whole forward from the
        current contents of the inputs with one kernel launch (rk_din_forward_plan /
        rk_din_plan_launch) and returns the same (prob, logit, l2_reg) tensors each time.  Like a
        captured graph it binds the current weights: prepare again after changing them."""
        if self.training:
            raise RuntimeError("DIN.prepare: eval mode only (call .eval() first)")
        pl = self._plan(dense, category, sequence, target)
        if not pl["fused"]:
            raise RuntimeError("DIN.prepare: configuration outside rk_din_forward's envelope")
        B, dev = pl["B"], pl["dev"]
        w = self.att_weights.get(dev)
        if self.att_weights.mode != "frozen":
            raise RuntimeError("DIN.prepare: per-call interaction weights are redrawn every forward; "
                               "use interaction_weights='frozen'")
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        want_l2 = pl["want_l2"]
        l2_reg = torch.empty((), device=dev, dtype=torch.float32) if want_l2 else None
        packed = [PACKED.pin(l.linear.weight) for l in self._tail]  # never rewritten under the plan
        layers = [ops.make_mlp_layer(l.linear.weight, pk, **l.epilogue_kwargs()) for l, pk in zip(self._tail, packed)]
        head = ops.make_epilogue(head_w=self.output_layer.weight, head_b=self.output_layer.bias,
                                 head_logit=logit, head_prob=prob)
        img = self._att_image(w, pl["H"])
        keep = (pl, w, img, packed, [l.epilogue_kwargs() for l in self._tail], logit, prob, l2_reg,
                self.embeddings[SEQ_KEY].weight)
        plan = ops.din_forward_plan(pl["segs"], pl["width"], pl["q_col"], pl["att_col"],
                                    self.embeddings[SEQ_KEY].weight, pl["seq"], pl["seq_len"], pl["H"], w,
                                    self.use_softmax, layers, head, B, dev, l2_col0=pl["cat_col0"],
                                    l2_scale=float(self.l2_lambda), l2_out=l2_reg, att_image=img, keep=keep)
        out = (prob, logit, l2_reg if want_l2 else 0.0)

        def run():
            plan.launch()
            return out
        run.plan = plan
        return run

    def fused_kernel_launcher(self, dense, category, sequence, target):
        """Zero-argument re-launch of this forward's rk_din_forward kernel (no l2 finish), for
        kernel-level timing (bench.py roofline)."""
        pl = self._plan(dense, category, sequence, target)
        if not pl["fused"]:
            raise RuntimeError("DIN configuration outside rk_din_forward's envelope")
        w = self.att_weights.get(pl["dev"])
        logit = torch.empty(pl["B"], 1, device=pl["dev"])
        prob = torch.empty_like(logit)
        return lambda: self._launch_fused(pl, w, logit, prob, None)

    def _eager_eval(self, dense, category, sequence, target):
        """The fused eval forward through the EagerCalls cache (see common.EagerCalls): on a hit
        one rk_din_forward call with fresh outputs (and the per-call H2 weights) patched in; None
        when the fused path does not apply."""
        if not common.EAGER_CACHE:
            return None
        try:
            dense_cols = list(dense.values())
            cats = [category[n] for n in self.embeddings if n in category]
            ins = dense_cols + cats + [target["feedid"], sequence[SEQ_KEY], sequence[f"{SEQ_KEY}_length"]]
        except (KeyError, TypeError, AttributeError):
            return None
        if not all(isinstance(t, torch.Tensor) for t in ins) or ins[0].device.type != "cuda":
            return None
        dev = ins[0].device
        stream = ops._lib.raw_stream(dev)
        calls = self.__dict__.setdefault("_eager", common.EagerCalls())
        key = calls.key(self, ins, stream, (self.att_weights.mode, tuple(dense), tuple(category)))
        if calls.get(key) is None and self._eager_build(dense, category, sequence, target, key, calls) is None:
            return None
        w = self.att_weights.get(dev)  # per-call mode: the reference's draws, once per forward
        args, head, B, want_l2, H, _keep = calls.get(key)
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        l2_reg = torch.empty((), device=dev, dtype=torch.float32) if want_l2 else 0.0
        head.head_logit = logit.data_ptr()
        head.head_prob = prob.data_ptr()
        img = self._att_image(w, H)
        args[14:20] = [t.data_ptr() for t in w]
        args[27] = l2_reg.data_ptr() if want_l2 else None
        args[28] = img.data_ptr()
        rc = ops._lib.load().rk_din_forward_ex(*args, stream)
        if rc == ops._lib.RK_ERR_UNSUPPORTED:  # e.g. past the kernel's LDS budget: the unfused path
            self._mark_unfusable(sequence[SEQ_KEY].shape[1], H)
            calls._d.pop(key, None)
            return None
        ops.check(rc, "rk_din_forward")
        return prob, logit, l2_reg

    def _mark_unfusable(self, T, H):
        """rk_din_forward refused this shape (RK_ERR_UNSUPPORTED, e.g. its LDS carve past 160 KiB with
        wide fcn layers): later forwards of the shape take the unfused launches."""
        width = None
        for l in self._tail[:1]:
            width = l.linear.in_features
        self.__dict__.setdefault("_unfusable", set()).add((width, T, H))

    def _eager_build(self, dense, category, sequence, target, key, calls):
        if not all(t.dtype == torch.int64 for t in list(category.values()) + [target["feedid"]] + list(sequence.values())):
            return None  # conversions make new tensors per call: the uncached path
        pl = self._plan(dense, category, sequence, target)
        if not pl["fused"] or pl["seq"].data_ptr() != sequence[SEQ_KEY].data_ptr():
            return None
        B, dev, H = pl["B"], pl["dev"], pl["H"]
        want_l2 = pl["want_l2"]
        packed = [PACKED(l.linear.weight) for l in self._tail]
        layers = [ops.make_mlp_layer(l.linear.weight, pk, **l.epilogue_kwargs()) for l, pk in zip(self._tail, packed)]
        head = ops.make_epilogue(head_w=self.output_layer.weight, head_b=self.output_layer.bias)
        zero = [torch.zeros(1, device=dev)] * 6  # placeholder H2 pointers, patched per call
        args, keep = ops._din_forward_args(pl["segs"], pl["width"], pl["q_col"], pl["att_col"],
                                           self.embeddings[SEQ_KEY].weight, pl["seq"], pl["seq_len"], H, zero,
                                           self.use_softmax, layers, head, B, dev, l2_col0=pl["cat_col0"],
                                           l2_scale=float(self.l2_lambda), l2_out=zero[0] if want_l2 else None,
                                           att_image=zero[0])
        # phase B's epilogue image packed once per entry (the key covers every parameter's
        # version) and copied into LDS by the kernel (rk_din_forward_ex), as a prepared plan does
        epi = ops.pack_epilogue_image(args[21], args[22], args[2], dev)
        # the entry keeps what its argument block points into (segment / layer arrays, packed
        # images, the l2 workspace) but not the caller's input tensors: the key's address, shape
        # and stride check already makes the raw input pointers valid on a hit
        return calls.put(key, (list(args) + [ops.ptr(epi)], head, B, want_l2, H, (keep, packed, layers, epi)))

    def forward(self, dense, category, sequence, target):
        tgt = target.get("feedid", None) if isinstance(target, dict) else None
        if not self.training and isinstance(tgt, torch.Tensor) and tgt.shape[0] == 0:
            # an empty batch: the reference still draws its attention MLP (din.py:61-67), and its l2
            # term is l2_lambda times the mean of no norms, NaN (din.py:319-322)
            dev = ops.require_gpu(tgt, "target['feedid']").device
            self.att_weights.get(dev)
            prob, logit = common.empty_rows(dev, 2)
            want_l2 = self.mini_batch_aware_regularization and self.l2_lambda > 0
            return prob, logit, (torch.full((), float("nan"), device=dev) if want_l2 else 0.0)
        if not self.training:
            out = self._eager_eval(dense, category, sequence, target)
            if out is not None:
                return out
        if self.training and not (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())):
            check_eval(self)  # a train-mode forward without autograd is not implemented
        pl = self._plan(dense, category, sequence, target)
        if self.training:  # Dice/BatchNorm batch statistics, Dropout, HIP backward (rankops.train)
            if self.embeddings[SEQ_KEY].embedding_dim != pl["H"]:
                raise NotImplementedError("rankops DIN training: target and history embeddings must share a width")
            prob, logit, l2 = train.din_train_forward(self, pl, self.att_weights.get(pl["dev"]))
            return prob, logit, (l2 if pl["want_l2"] else 0.0)
        B, dev, segs, H = pl["B"], pl["dev"], pl["segs"], pl["H"]
        cat_col0, q_col, att_col, width = pl["cat_col0"], pl["q_col"], pl["att_col"], pl["width"]
        seq, seq_len = pl["seq"], pl["seq_len"]
        T = seq.shape[1]
        w = self.att_weights.get(dev)
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        want_l2 = self.mini_batch_aware_regularization and self.l2_lambda > 0

        if pl["fused"]:
            # the whole forward in one launch (rk_din_forward)
            l2_reg = torch.empty((), device=dev, dtype=torch.float32) if want_l2 else 0.0
            try:
                self._launch_fused(pl, w, logit, prob, l2_reg)
                return prob, logit, l2_reg
            except ops._lib.RankOpsError as e:
                if getattr(e, "code", None) != ops._lib.RK_ERR_UNSUPPORTED:
                    raise
                self._mark_unfusable(T, H)

        row = torch.empty(B, width, device=dev, dtype=torch.float32)
        ops.concat_gather(segs, B, row)
        ops.din_attention(ops._lib.fptr(row, q_col), width, self.embeddings[SEQ_KEY].weight, seq, seq_len, T, H, w,
                          self.use_softmax, ops._lib.fptr(row, att_col), width, B, dev)
        run_tail(row, self._tail, self.output_layer, {}, logit, prob)

        l2_reg = 0.0
        if want_l2:
            l2_reg = torch.empty((), device=dev, dtype=torch.float32)
            ops.row_l2norm_mean(row, cat_col0, width - cat_col0, float(self.l2_lambda), l2_reg)
        return prob, logit, l2_reg
