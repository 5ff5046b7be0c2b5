"""BST (Behavior Sequence Transformer) on the rankops engine — drop-in for algorithm/BST/bst.py.

`BSTModel(vocab_dir, hidden_units=[512,256,128], dropout_rate=0.1, batch_norm=True, d_model=16,
nhead=4, num_transformer_blocks=1, max_seq_length=50, pooling_method='sum')` keeps the
reference constructor, creation order, state_dict keys (`embeddings.*`,
`transformer_blocks.N.{position_embedding,w_q,w_k,w_v,w_o,norm1,norm2,ffn.0,ffn.3}.*`,
`dnn.N.*`; bst.py:162-214) and `forward(dense, category, seq_feedid, seq_length) ->
(probabilities, logits)` (bst.py:216-247).  The reference hard-codes the transformer width to
16 (bst.py:188,192,201); here `d_model` sets it (default 16 = the reference) so the
benchmark's d_model=128 runs through the same class.

Per transformer block (bst.py:66-91):
  rk_linear   [Q|K] = (x + pos) W_{q,k}^T + b          (positions added in the A-tile loader)
  rk_linear   V = x W_v^T + b_v
  rk_bst_attention   masked softmax(QK^T/sqrt(d_h)) V per head (-inf mask, NaN for empty rows)
  rk_linear   out1 = LN1((x + pos) + ctx W_o^T + b_o)    (residual + LayerNorm in the epilogue)
  rk_linear   f = LeakyReLU(out1 W_1^T + b_1)
  rk_linear   out = LN2(out1 + f W_2^T + b_2); the last block sums (or averages) the T rows of
              each sample straight into the DNN input row (bst.py:238-241)
then rk_concat_gather for [dense | category] and the DNN on rk_linear with the final Linear +
sigmoid fused.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import common, ops, train
from .common import EngineModule, Layer, Packed, check_eval, run_tail, table_rows

FIELDS = ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list")


def load_vocabulary(vocab_file):
    import os
    if not os.path.exists(vocab_file):
        return []
    with open(vocab_file, 'r') as f:
        return [line.strip() for line in f]


class BSTTransformer(EngineModule):
    """Transformer block with the reference's parameters (bst.py:42-64)."""

    def __init__(self, d_model, nhead, max_len, dropout=0.1):
        super().__init__()
        self.d_model = d_model
        self.nhead = nhead
        self.position_embedding = nn.Embedding(max_len, d_model)
        self.w_q = nn.Linear(d_model, d_model)
        self.w_k = nn.Linear(d_model, d_model)
        self.w_v = nn.Linear(d_model, d_model)
        self.w_o = nn.Linear(d_model, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.dropout = nn.Dropout(dropout)
        self.ffn = nn.Sequential(
            nn.Linear(d_model, d_model),
            nn.LeakyReLU(negative_slope=0.01),
            nn.Dropout(dropout),
            nn.Linear(d_model, d_model),
        )
        self._wqk = Packed()
        self._bqk = Packed()

    def forward(self, queries, keys, values, key_padding_mask=None):
        """BSTTransformer.forward(queries, keys, values, key_padding_mask=None) (bst.py:66-91):
        queries/keys/values [B, T, d]; key_padding_mask [B, T] bool (True = padding key) or None.
        Eval semantics (Dropout identity).  rk_linear for Q (queries + positions), K (keys +
        positions), V, W_o + residual + LayerNorm1 and the FFN + residual + LayerNorm2, and
        rk_bst_attention_masked in between; a row whose keys are all masked gives NaN, as torch's
        softmax over an all -inf row does."""
        check_eval(self)
        queries = ops.as_f32(queries, "queries")
        keys = ops.as_f32(keys, "keys")
        values = ops.as_f32(values, "values")
        if queries.dim() != 3 or keys.shape != queries.shape or values.shape != queries.shape:
            raise ValueError(f"BSTTransformer: queries {tuple(queries.shape)}, keys {tuple(keys.shape)} and values "
                             f"{tuple(values.shape)} must all be [batch, seq_len, d_model]")
        B, T, d = queries.shape
        if d != self.d_model:
            raise ValueError(f"BSTTransformer: d_model {self.d_model}, inputs have {d}")
        pos = self.position_embedding.weight
        if T > pos.shape[0]:
            raise IndexError(f"BSTTransformer: sequence length {T} exceeds max_len {pos.shape[0]}")
        dev = queries.device
        out = torch.empty(B, T, d, device=dev, dtype=torch.float32)
        if B == 0:
            return out
        mask = None
        if key_padding_mask is not None:
            require = ops.require_gpu(key_padding_mask, "key_padding_mask")
            if require.dtype != torch.bool or tuple(require.shape) != (B, T):
                raise ValueError(f"BSTTransformer: key_padding_mask must be a bool [{B}, {T}] tensor, got "
                                 f"{require.dtype} {tuple(require.shape)}")
            mask = require.contiguous().view(torch.uint8)
        q2 = queries.reshape(B * T, d).contiguous()
        k2 = q2 if keys is queries else keys.reshape(B * T, d).contiguous()
        v2 = q2 if values is queries else values.reshape(B * T, d).contiguous()
        qkv = torch.empty(B * T, 3 * d, device=dev, dtype=torch.float32)
        if k2 is q2:  # self-attention: [W_q; W_k] as one GEMM with the positions added in the A loader
            ops.linear(q2, self._wqk(self.w_q.weight, self.w_k.weight), None, x_periodic=pos, x_period=T,
                       y_ptr=qkv.data_ptr(), ldy=3 * d, epilogue=ops.make_epilogue(bias=self._bqk(self.w_q.bias,
                                                                                                  self.w_k.bias)))
        else:
            ops.linear(q2, self.w_q.weight, None, x_periodic=pos, x_period=T, y_ptr=qkv.data_ptr(), ldy=3 * d,
                       epilogue=ops.make_epilogue(bias=self.w_q.bias))
            ops.linear(k2, self.w_k.weight, None, x_periodic=pos, x_period=T, y_ptr=ops._lib.fptr(qkv, d),
                       ldy=3 * d, epilogue=ops.make_epilogue(bias=self.w_k.bias))
        ops.linear(v2, self.w_v.weight, None, y_ptr=ops._lib.fptr(qkv, 2 * d), ldy=3 * d,
                   epilogue=ops.make_epilogue(bias=self.w_v.bias))
        ctx = torch.empty(B * T, d, device=dev, dtype=torch.float32)
        ops.bst_attention_masked(qkv, B, T, d, self.nhead, mask, ctx)
        self._tail(ctx, q2, pos, T, out.view(B * T, d))
        return out

    def _tail(self, ctx, x, pos, T, out, pool_out_ptr=None, ld_pool=0, pool_mean=False, seq_length=None):
        """out1 = LN1((x + pos) + ctx W_o^T + b_o); out = LN2(out1 + FFN(out1)) (bst.py:86-90),
        optionally summed / averaged per sample into pool_out_ptr (bst.py:238-241)."""
        d = self.d_model
        out1 = torch.empty(x.shape[0], d, device=x.device, dtype=torch.float32)
        ops.linear(ctx, self.w_o.weight, out1, epilogue=ops.make_epilogue(
            bias=self.w_o.bias, residual=x, ld_residual=x.stride(0), residual_periodic=pos, residual_period=T,
            has_ln=1, ln_gamma=self.norm1.weight, ln_beta=self.norm1.bias, ln_eps=self.norm1.eps))
        f1 = torch.empty(x.shape[0], d, device=x.device, dtype=torch.float32)
        ops.linear(out1, self.ffn[0].weight, f1, epilogue=ops.make_epilogue(
            bias=self.ffn[0].bias, act="leaky", slope=self.ffn[1].negative_slope))
        ep = dict(bias=self.ffn[3].bias, residual=out1, ld_residual=out1.stride(0), has_ln=1,
                  ln_gamma=self.norm2.weight, ln_beta=self.norm2.bias, ln_eps=self.norm2.eps)
        if pool_out_ptr is not None:
            ep.update(pool_out=pool_out_ptr, ld_pool=ld_pool, pool_rows=T, pool_mean=1 if pool_mean else 0,
                      pool_len=seq_length)
        ops.linear(f1, self.ffn[3].weight, out, epilogue=ops.make_epilogue(**ep))
        return out

    def run(self, x: torch.Tensor, B: int, T: int, seq_length: torch.Tensor, out: torch.Tensor = None,
            pool_out_ptr: int = None, ld_pool: int = 0, pool_mean: bool = False):
        """x: [B*T, d] (queries = keys = values).  Writes the block output to `out`, or pools it
        per sample into pool_out_ptr when given."""
        d = self.d_model
        dev = x.device
        pos = self.position_embedding.weight
        if T > pos.shape[0]:
            raise IndexError(f"BSTTransformer: sequence length {T} exceeds max_len {pos.shape[0]}")
        qkv = torch.empty(B * T, 3 * d, device=dev, dtype=torch.float32)
        wqk = self._wqk(self.w_q.weight, self.w_k.weight)
        bqk = self._bqk(self.w_q.bias, self.w_k.bias)
        ops.linear(x, wqk, None, x_periodic=pos, x_period=T, y_ptr=qkv.data_ptr(), ldy=3 * d,
                   epilogue=ops.make_epilogue(bias=bqk))
        ops.linear(x, self.w_v.weight, None, y_ptr=ops._lib.fptr(qkv, 2 * d), ldy=3 * d,
                   epilogue=ops.make_epilogue(bias=self.w_v.bias))
        ctx = torch.empty(B * T, d, device=dev, dtype=torch.float32)
        ops.bst_attention(qkv, B, T, d, self.nhead, seq_length, ctx)
        return self._tail(ctx, x, pos, T, out, pool_out_ptr, ld_pool, pool_mean, seq_length)


class BSTModel(EngineModule):
    def __init__(self, vocab_dir, hidden_units=[512, 256, 128], dropout_rate=0.1, batch_norm=True, d_model=16,
                 nhead=4, num_transformer_blocks=1, max_seq_length=50, pooling_method='sum', *,
                 vocab_sizes=None):
        super().__init__()
        self.vocab_sizes = {f: table_rows(vocab_dir, f, vocab_sizes) for f in FIELDS}
        self.num_dense_features = 16
        self.d_model = d_model
        self.embeddings = nn.ModuleDict({
            'userid': nn.Embedding(self.vocab_sizes['userid'], 16),
            'device': nn.Embedding(self.vocab_sizes['device'], 2),
            'authorid': nn.Embedding(self.vocab_sizes['authorid'], 4),
            'bgm_song_id': nn.Embedding(self.vocab_sizes['bgm_song_id'], 4),
            'bgm_singer_id': nn.Embedding(self.vocab_sizes['bgm_singer_id'], 4),
            'manual_tag_list': nn.Embedding(self.vocab_sizes['manual_tag_list'], 4),
            'feedid': nn.Embedding(self.vocab_sizes['feedid'], d_model),
        })
        self.transformer_blocks = nn.ModuleList([
            BSTTransformer(d_model=d_model, nhead=nhead, max_len=max_seq_length + 1, dropout=dropout_rate)
            for _ in range(num_transformer_blocks)
        ])
        self.batch_norm = batch_norm
        self.dropout_rate = dropout_rate
        self.pooling_method = pooling_method
        category_emb_dim = 16 + 2 + 4 + 4 + 4 + 4
        layers = []
        self._tail = []
        width = self.num_dense_features + category_emb_dim + d_model
        for h in hidden_units:
            lin = nn.Linear(width, h)
            layers.append(lin)
            bn = None
            if batch_norm:
                bn = nn.BatchNorm1d(h)
                layers.append(bn)
            act = nn.LeakyReLU(negative_slope=0.01)
            layers.append(act)
            if dropout_rate > 0:
                layers.append(nn.Dropout(dropout_rate))
            self._tail.append(Layer(lin, pre_bn=bn, act="leaky", slope=act.negative_slope))
            width = h
        layers.append(nn.Linear(width, 1))
        self.dnn = nn.Sequential(*layers)
        self._dropout = train.DropoutStreams()

    def forward(self, dense, category, seq_feedid, seq_length):
        if self.training and not (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())):
            check_eval(self)  # a train-mode forward without autograd is not implemented
        dense = ops.as_f32(dense, "dense")
        seq_feedid = ops.as_index(seq_feedid, "seq_feedid").contiguous()
        seq_length = ops.as_index(seq_length, "seq_length")
        if not self.training and seq_feedid.shape[0] == 0:
            return common.empty_rows(dense.device, 2)
        if self.training:  # Dropout in the blocks and the dnn, BatchNorm batch statistics, HIP backward
            for blk in self.transformer_blocks:
                if seq_feedid.shape[1] > blk.position_embedding.num_embeddings:
                    raise IndexError(f"BSTTransformer: sequence length {seq_feedid.shape[1]} exceeds max_len "
                                     f"{blk.position_embedding.num_embeddings}")
            return train.bst_train_forward(self, dense.contiguous(), category, seq_feedid, seq_length)
        B, T = seq_feedid.shape
        dev = dense.device
        d = self.d_model
        # DNN input row: [dense | category embeddings | pooled transformer output]
        segs = [ops.dense_segment(dense, self.num_dense_features, 0)]
        col = self.num_dense_features
        for name, emb in self.embeddings.items():
            if name in category:
                idx = ops.as_index(category[name], f"category[{name!r}]")
                segs.append(ops.table_segment(emb.weight, idx, col))
                col += emb.embedding_dim
        width = col + d
        nblk = len(self.transformer_blocks)
        row = None
        if nblk == 0:
            row = torch.empty(B, width, device=dev, dtype=torch.float32)
            ops.concat_gather(segs, B, row)
            # no transformer blocks (bst.py:228-235 leaves transformer_output = seq_emb): gather the
            # history rows, then sum / mean pooling over all T positions into the DNN row
            seq = torch.empty(B * T, d, device=dev, dtype=torch.float32)
            ops.concat_gather([ops.table_segment(self.embeddings['feedid'].weight, seq_feedid.view(-1), 0)], B * T,
                              seq)
            ops.bst_pool(seq, B, T, seq_length, self.pooling_method != 'sum', row, col)
            logits = torch.empty(B, 1, device=dev, dtype=torch.float32)
            probs = torch.empty(B, 1, device=dev, dtype=torch.float32)
            run_tail(row, self._tail, self.dnn[-1], {}, logits, probs)
            return probs, logits
        for blk in self.transformer_blocks:
            if T > blk.position_embedding.num_embeddings:
                raise IndexError(f"BSTTransformer: sequence length {T} exceeds max_len "
                                 f"{blk.position_embedding.num_embeddings}")
        blocks = self._fused_blocks(T)
        if blocks is not None and d == 16 and common.FUSED_BST_FWD:
            # the whole forward in one launch (rk_bst_small_forward): row gather, blocks, pooling,
            # DNN tail and head; outside its envelope the three launches below
            logits = torch.empty(B, 1, device=dev, dtype=torch.float32)
            probs = torch.empty(B, 1, device=dev, dtype=torch.float32)
            mls = [ops.make_mlp_layer(l.linear.weight, common.PACKED(l.linear.weight), **l.epilogue_kwargs())
                   for l in self._tail]
            head = ops.make_epilogue(head_w=self.dnn[-1].weight, head_b=self.dnn[-1].bias, head_logit=logits,
                                     head_prob=probs)
            if ops.bst_small_forward(segs, col, self.embeddings['feedid'].weight, seq_feedid, seq_length,
                                     self.transformer_blocks[0].nhead, blocks, self.pooling_method != 'sum', mls,
                                     head):
                return probs, logits
        row = torch.empty(B, width, device=dev, dtype=torch.float32)
        ops.concat_gather(segs, B, row)
        if blocks is not None:
            # every block + pooling in one launch, activations in LDS (rk_bst_forward_blocks)
            packed = d == 128
            ops.bst_forward_blocks(self.embeddings['feedid'].weight, seq_feedid, seq_length, d,
                                   self.transformer_blocks[0].nhead, self._packed_blocks(blocks) if packed else blocks,
                                   ops._lib.fptr(row, col), width, self.pooling_method != 'sum', packed=packed)
        else:
            self._run_blocks(row, col, width, seq_feedid, seq_length, B, T)
        logits = torch.empty(B, 1, device=dev, dtype=torch.float32)
        probs = torch.empty(B, 1, device=dev, dtype=torch.float32)
        run_tail(row, self._tail, self.dnn[-1], {}, logits, probs)
        return probs, logits

    def prepare(self, dense, category, seq_feedid, seq_length):
        """An eval forward bound to these input tensors (as DIN.prepare / DCNModel.prepare: the
        single-kernel analogue of capturing the forward in a hipGraph) at the reference script's
        d_model 16: returns `run()` that recomputes the whole forward from the current contents of
        the inputs with one rk_bst_small_forward launch and returns the same (prob, logit) tensors
        each time.  Binds the current weights (repack-free: the packed tail images are pinned).  Index
        tensors must be int64 and seq_feedid contiguous (bound by address, never copied)."""
        if self.training:
            raise RuntimeError("BSTModel.prepare: eval mode only (call .eval() first)")
        dense = ops.as_f32(dense, "dense")
        seq_feedid = ops.bound_index(seq_feedid, "seq_feedid", contiguous=True)
        seq_length = ops.bound_index(seq_length, "seq_length")
        B, T = seq_feedid.shape
        dev = dense.device
        blocks = self._fused_blocks(T) if self.transformer_blocks else None
        if blocks is None or self.d_model != 16 or not common.FUSED_BST_FWD:
            raise RuntimeError("BSTModel.prepare: configuration outside rk_bst_small_forward's envelope")
        segs = [ops.dense_segment(dense, self.num_dense_features, 0)]
        col = self.num_dense_features
        idx_keep = []
        for name, emb in self.embeddings.items():
            if name in category:
                idx = ops.bound_index(category[name], f"category[{name!r}]")
                idx_keep.append(idx)
                segs.append(ops.table_segment(emb.weight, idx, col))
                col += emb.embedding_dim
        logits = torch.empty(B, 1, device=dev, dtype=torch.float32)
        probs = torch.empty(B, 1, device=dev, dtype=torch.float32)
        packed = [common.PACKED(l.linear.weight) for l in self._tail]
        for l in self._tail:  # the images the launch binds are never rewritten in place under it
            common.PACKED.pin(l.linear.weight)
        epis = [l.epilogue_kwargs() for l in self._tail]  # folded BatchNorm tensors: kept alive below
        mls = [ops.make_mlp_layer(l.linear.weight, pk, **ek) for l, pk, ek in zip(self._tail, packed, epis)]
        head = ops.make_epilogue(head_w=self.dnn[-1].weight, head_b=self.dnn[-1].bias, head_logit=logits,
                                 head_prob=probs)
        args = ops.bst_small_forward_args(segs, col, self.embeddings['feedid'].weight, seq_feedid, seq_length,
                                          self.transformer_blocks[0].nhead, blocks, self.pooling_method != 'sum',
                                          mls, head)
        fn, out = ops._lib.load().rk_bst_small_forward, (probs, logits)
        rc = fn(*args)
        if rc == ops._lib.RK_ERR_UNSUPPORTED:
            raise RuntimeError("BSTModel.prepare: configuration outside rk_bst_small_forward's envelope")
        ops.check(rc, "rk_bst_small_forward")

        def run():
            ops.check(fn(*args), "rk_bst_small_forward")
            return out
        run.keep = (args, head, mls, packed, epis, blocks, segs, idx_keep, dense, seq_feedid, seq_length, category)
        return run

    def blocks_kernel_launcher(self, seq_feedid, seq_length):
        """Zero-argument re-launch of this forward's rk_bst_forward_blocks kernel (every block +
        pooling) into a scratch DNN row, for kernel-level timing (bench.py BST roofline)."""
        seq_feedid = ops.bound_index(seq_feedid, "seq_feedid", contiguous=True)
        seq_length = ops.bound_index(seq_length, "seq_length")
        B, T = seq_feedid.shape
        blocks = self._fused_blocks(T)
        if blocks is None or not self.transformer_blocks:
            raise RuntimeError("BST configuration outside rk_bst_forward_blocks' envelope")
        d = self.d_model
        row = torch.empty(B, d, device=seq_feedid.device, dtype=torch.float32)
        packed = d == 128
        if packed:
            blocks = self._packed_blocks(blocks)
        return lambda: ops.bst_forward_blocks(self.embeddings['feedid'].weight, seq_feedid, seq_length, d,
                                              self.transformer_blocks[0].nhead, blocks, ops._lib.fptr(row, 0), d,
                                              self.pooling_method != 'sum', packed=packed)

    @staticmethod
    def _packed_blocks(blocks):
        """_fused_blocks' parameters with the six d-128 projection weights (wq, wk, wv, wo, ffn.0,
        ffn.3) replaced by their rk_bst_pack_block_weight images (cached per weight version)."""
        out = []
        for ts, sc in blocks:
            ts = list(ts)
            for k in (1, 3, 5, 7, 9, 11):
                ts[k] = common.BST_PACKED(ts[k])
            out.append((tuple(ts), sc))
        return out

    def _fused_blocks(self, T):
        """Parameters for rk_bst_forward_blocks, or None outside its envelope: d_model 128 with 4
        heads (bst_block_kernel) or the reference script's d_model 16 with 1/2/4/8 heads
        (bst_small_kernel); T <= 64, <= 4 blocks, contiguous 16-B aligned fp32 parameters."""
        blks = self.transformer_blocks
        d = self.d_model
        heads_ok = (lambda h: h == 4) if d == 128 else (lambda h: h in (1, 2, 4, 8))
        if not (common.FUSED_BST and d in (16, 128) and 1 <= T <= 64 and len(blks) <= 4
                and self.embeddings['feedid'].weight.stride(0) == d
                and self.embeddings['feedid'].weight.data_ptr() % 16 == 0
                and all(heads_ok(b.nhead) for b in blks)):
            return None
        out = []
        for b in blks:
            ts = (b.position_embedding.weight, b.w_q.weight, b.w_q.bias, b.w_k.weight, b.w_k.bias, b.w_v.weight,
                  b.w_v.bias, b.w_o.weight, b.w_o.bias, b.ffn[0].weight, b.ffn[0].bias, b.ffn[3].weight,
                  b.ffn[3].bias, b.norm1.weight, b.norm1.bias, b.norm2.weight, b.norm2.bias)
            if any(t.dtype != torch.float32 or not t.is_contiguous() or t.data_ptr() % 16 for t in ts):
                return None
            out.append((ts, (b.norm1.eps, b.norm2.eps, b.ffn[1].negative_slope)))
        return out

    def _run_blocks(self, row, col, width, seq_feedid, seq_length, B, T):
        """Per-layer path: gathered sequence in HBM, rk_linear x5 + rk_bst_attention per block."""
        d = self.d_model
        dev = row.device
        # behaviour sequence: x[b*T + t] = feedid_table[seq_feedid[b, t]]
        x = torch.empty(B * T, d, device=dev, dtype=torch.float32)
        flat = seq_feedid.view(-1)
        ops.concat_gather([ops.table_segment(self.embeddings['feedid'].weight, flat, 0)], B * T, x)
        nblk = len(self.transformer_blocks)
        for i, blk in enumerate(self.transformer_blocks):
            if i == nblk - 1:
                blk.run(x, B, T, seq_length, pool_out_ptr=ops._lib.fptr(row, col), ld_pool=width,
                        pool_mean=self.pooling_method != 'sum')
            else:
                x = blk.run(x, B, T, seq_length, out=torch.empty_like(x))
