"""Table-sharded DeepFM across the GPUs of one node (BASELINE configs[4]: 1e8 embedding rows,
global batch 65536) — embedding lookup exchanged with two RCCL all-to-alls over xGMI.

Layout: table-wise sharding.  Field f (in DeepFM field order) lives on rank f % P with both its
second-order [V_f, D] and first-order [V_f, 1] tables; the dense layers are replicated.  Each
rank holds a data-parallel slice of B_l samples with the indices of all F fields.  One forward:

  1. index exchange   all_to_all_single: rank r receives, from every source s, the indices of
                      r's fields for s's samples, laid out [s][b][f_r] (int32 on the wire while
                      every table has < 2^31 rows — configs[4]: 3.3M per field — else int64)
  2. local gather     one rk_concat_gather from r's packed tables (rk_fm_pack_table: per field
                      one [V_f, RS] table, the D second-order floats at 0..D-1 and the
                      first-order weight at D, RS = D + 1 rounded up to 4 floats so every row
                      stays 16-B aligned) -> rows [s][b][f_r][RS], one contiguous read per row
  3. row exchange     all_to_all_single back: each source gets [r][b][f_r][RS] from every owner
  4. FM + MLP         rk_deepfm_forward over the received rows, read in place as dense blocks of
                      packed rows (field order restored through out_col = f * D): fm1, fm2, the
                      deep layers and the head in one launch, the [B, F*D] deep input never
                      written to HBM (configs[4]'s shape; other shapes: rk_fm_linear_packed,
                      then the streamed MLP tail — DeepFM's two-launch forward)

At P > 1 the index exchange covers the whole local batch (one rk_shard_pack_indices launch, one
all-to-all), then steps 2-4 run per chunk of the local batch (run_steps): each chunk's gather
(rk_shard_gather_rows, straight from the received int32 indices) feeds a row all-to-all that is
issued asynchronously and overlaps the next chunk's gather and the previous chunk's FM + tail.
At P = 1 there is nothing to exchange: the forward is rk_deepfm_forward over the packed tables,
i.e. `DeepFM.forward` on the same weights.
The exchange volume per rank and step is B_l * F * (4 + 4 * RS) bytes (int32 indices), (P-1)/P of
it on the wire, with the packed rows; the split wire format (round 5, `wire`, the default where
the one-launch forward applies) sends D floats per (sample, field) straight from the [V, D]
nn.Embedding weight plus one first-order partial sum per (sample, owner): B_l * (F * (4 + 4 * D) +
4 * P) bytes, and the owner reads one 128-B line per row instead of the packed row's two.  Rows travel at RS = 36 floats (144 B, 132 live): the receiver's fused front end
reads them in place with 16-B loads, which a 132-B stride would misalign for three rows in four,
and the row exchange overlaps the next chunk's gather.  Reference: DeepFM.forward, deepfm.py:121-151 (the reference is single-device; the
sharding is the MI355X build's own).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from . import ops
from .common import EngineModule, Layer, PackedFMTable, check_eval, run_tail


def row_stride(dim: int) -> int:
    return (dim + 1 + 3) // 4 * 4


def field_owner(num_fields: int, world: int):
    """Field index -> owning rank (round robin: 30 fields on 8 ranks = 4/4/4/4/4/4/3/3)."""
    return [f % world for f in range(num_fields)]


class ShardedDeepFM(EngineModule):
    def __init__(self, field_rows: dict, embedding_dim=32, hidden_units=None, dropout_rate=0.1, batch_norm=True,
                 *, group=None, rank: int = None, world_size: int = None):
        super().__init__()
        if hidden_units is None:
            hidden_units = [512, 256, 128]
        self.group = group
        if world_size is None:
            world_size = dist.get_world_size(group) if dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.rank, self.world = rank, world_size
        self.fields = list(field_rows)
        self.field_rows = dict(field_rows)
        self.embedding_dim = embedding_dim
        self.owner = field_owner(len(self.fields), world_size)
        self.fields_of = [[f for i, f in enumerate(self.fields) if self.owner[i] == r] for r in range(world_size)]
        self.local_fields = self.fields_of[rank]
        self.pipeline_chunks = 4  # exchange pipeline depth at P > 1 (chunk_bounds)
        # smallest chunk: 4096 samples keep the fused front end's 64 x 128 tiles on every CU
        # (rk_fm_linear_packed at 2048 rows leaves half the chip idle)
        self.min_chunk = 4096
        # all-to-all transport: None = torch.distributed.all_to_all_single on `group` (RCCL);
        # otherwise a callable (out, inp, out_splits, in_splits, async_op) -> out | (out, work)
        # with the same semantics (tests drive P shards in one process through an emulator)
        self.exchange_fn = None
        # index wire format: int32 while every table fits (the receiver widens before its gather)
        self.index_dtype = torch.int32 if max(self.field_rows.values()) < 2 ** 31 else torch.int64
        # gather + FM + first deep layer in one rk_fm_linear_packed launch (False: the three-launch
        # rk_fm_gather(_packed) + tiled first layer + tail path, kept for A/B)
        self.fused_front = True
        # ... and, where a plan is compiled for the shape (960 -> 512 -> 256 -> 128), the whole
        # forward in one rk_deepfm_forward launch (False: rk_fm_linear_packed + the tail)
        self.fused_whole = True
        # row-exchange wire format (round 5): "split" = each field's D second-order floats read from
        # the [V, D] nn.Embedding weight as they are (one 128-B line at D = 32) plus ONE first-order
        # value per (sample, owner) — the sum of the owner's fields' weights — received by
        # rk_deepfm_forward_fo; "packed" = the rk_fm_pack_table row, pad4(D + 1) floats per field.
        # split applies where the one-launch forward does (split_wire()); otherwise packed.
        self.wire = "split"
        self.first_order_embeddings = nn.ModuleDict({f: nn.Embedding(self.field_rows[f], 1)
                                                     for f in self.local_fields})
        self.second_order_embeddings = nn.ModuleDict({f: nn.Embedding(self.field_rows[f], embedding_dim)
                                                      for f in self.local_fields})
        self.deep_layers = nn.ModuleList()
        self._tail = []
        width = len(self.fields) * embedding_dim
        for unit in hidden_units:
            lin = nn.Linear(width, unit)
            self.deep_layers.append(lin)
            bn = None
            if batch_norm:
                bn = nn.BatchNorm1d(unit)
                self.deep_layers.append(bn)
            self.deep_layers.append(nn.ReLU())
            if dropout_rate > 0:
                self.deep_layers.append(nn.Dropout(dropout_rate))
            self._tail.append(Layer(lin, pre_bn=bn, act="relu"))
            width = unit
        self.deep_output_layer = nn.Linear(width, 1)
        self.final_layer = nn.Linear(3, 1)
        self._fm_packs = {f: PackedFMTable() for f in self.local_fields}

    def packed_table(self, f):
        """This rank's packed [V_f, RS] table of field f (cached per weight version)."""
        return self._fm_packs[f](self.second_order_embeddings[f].weight, self.first_order_embeddings[f].weight)

    @classmethod
    def from_deepfm(cls, model, *, group=None, rank=None, world_size=None):
        """Shard a full DeepFM's parameters: this rank keeps its fields' tables and all dense layers."""
        rows = {f: e.num_embeddings for f, e in model.second_order_embeddings.items()}
        hidden = [l.out_features for l in model.deep_layers if isinstance(l, nn.Linear)]
        bn = any(isinstance(l, nn.BatchNorm1d) for l in model.deep_layers)
        drop = any(isinstance(l, nn.Dropout) for l in model.deep_layers)
        with torch.device("meta"):
            sh = cls(rows, model.embedding_dim, hidden, 0.1 if drop else 0.0, bn, group=group, rank=rank,
                     world_size=world_size)
        sd = model.state_dict()
        mine = {k: v for k, v in sd.items()
                if not k.startswith(("first_order_embeddings.", "second_order_embeddings."))
                or k.split(".")[1] in sh.local_fields}
        sh = sh.to_empty(device=next(model.parameters()).device)
        sh.load_state_dict(mine, strict=True)
        return sh.eval()

    # ------------------------------------------------------------------ exchange steps

    def _exchange(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, async_op: bool = False):
        """all_to_all_single (RCCL on ROCm); with async_op the collective runs on the process
        group's stream and the returned work's wait() orders the caller's stream after it."""
        if self.world == 1:
            out.copy_(inp)
            return (out, None) if async_op else out
        if self.exchange_fn is not None:
            return self.exchange_fn(out, inp, out_splits, in_splits, async_op)
        work = dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group, async_op=async_op)
        return (out, work) if async_op else out

    def split_wire(self) -> bool:
        """Whether the row exchange uses the split format (config only: the same on every rank)."""
        D = self.embedding_dim
        widths = [l.linear.out_features for l in self._tail]
        return (self.wire == "split" and self.world > 1 and self.fused_front and self.fused_whole
                and self.index_dtype == torch.int32 and len(self._tail) >= 2 and len(self.fields) <= 32
                and 4 <= D <= 256 and D & (D - 1) == 0 and ops.deepfm_whole_plan(len(self.fields) * D, widths))

    def _block(self, B: int, F_r: int) -> int:
        """Floats of one owner's row block for B samples of F_r of its fields (an owner with no
        fields, world > fields, sends nothing: no receiver reads an empty owner's partials)."""
        if F_r == 0:
            return 0
        if self.split_wire():
            return B * F_r * self.embedding_dim + (B + 3) // 4 * 4
        return B * F_r * row_stride(self.embedding_dim)

    def index_splits(self, B_l: int):
        """(output_split_sizes, input_split_sizes) of the index all-to-all, in int64 elements."""
        F_me = len(self.local_fields)
        return [B_l * F_me] * self.world, [B_l * len(self.fields_of[r]) for r in range(self.world)]

    def row_splits(self, B_l: int):
        """(output_split_sizes, input_split_sizes) of the row all-to-all, in floats."""
        F_me = len(self.local_fields)
        return [self._block(B_l, len(self.fields_of[r])) for r in range(self.world)], [self._block(B_l, F_me)] * self.world

    def pack_indices(self, category: dict) -> torch.Tensor:
        """Send buffer of step 1: [r][b][f_r] index blocks in index_dtype (on the GPU with int32:
        one rk_shard_pack_indices launch)."""
        first = category[self.fields[0]]
        if self.index_dtype == torch.int32 and first.is_cuda and all(
                category[f].dtype == torch.int64 and category[f].stride(0) == 1 for f in self.fields):
            return self._pack_indices_kernel(category, first.shape[0])
        blocks = []
        for r in range(self.world):
            fr = self.fields_of[r]
            if fr:
                blocks.append(torch.stack([category[f] for f in fr], 1).reshape(-1))
        if not blocks:
            return torch.empty(0, dtype=self.index_dtype, device=self._device())
        idx = torch.cat(blocks)
        if self.index_dtype == torch.int32:  # as rk_shard_pack_indices: never wrap to a valid row
            idx = torch.where((idx >= 0) & (idx <= 2 ** 31 - 1), idx, torch.full_like(idx, -1))
        return idx.to(self.index_dtype)

    def _pack_indices_kernel(self, category: dict, B: int) -> torch.Tensor:
        import ctypes
        n = len(self.fields)
        ptrs, base, stride = (ctypes.c_void_p * n)(), (ctypes.c_int64 * n)(), (ctypes.c_int32 * n)()
        q, start = 0, 0
        for r in range(self.world):
            fr = self.fields_of[r]
            for j, f in enumerate(fr):
                ptrs[q], base[q], stride[q] = category[f].data_ptr(), B * start + j, len(fr)
                q += 1
            start += len(fr)
        out = torch.empty(B * n, dtype=torch.int32, device=category[self.fields[0]].device)
        lib = ops._lib.load()
        ops._lib.ensure_device(out.device)
        ops.check(lib.rk_shard_pack_indices(ptrs, base, stride, n, B, out.data_ptr(), ops._lib.stream_of(out)),
                  "rk_shard_pack_indices")
        return out

    def exchange_indices(self, category: dict, B_l: int, async_op: bool = False):
        """Step 1: send [r][b][f_r] index blocks; receive [s][b][f_me]."""
        send = self.pack_indices(category)
        out_s, in_s = self.index_splits(B_l)
        recv = torch.empty(sum(out_s), dtype=self.index_dtype, device=send.device)
        return self._exchange(recv, send, out_s, in_s, async_op)

    def gather_rows(self, recv_idx: torch.Tensor, B_src: int, b0: int, bc: int) -> torch.Tensor:
        """Step 2 for samples [b0, b0 + bc) of every source: rows [s][b'][f_me][RS] from this rank's
        packed tables at the received indices (recv_idx: [s][B_src][f_me] as exchanged).  int32:
        one rk_shard_gather_rows launch; int64: rk_concat_gather over the chunk's copy."""
        RS, F_me = row_stride(self.embedding_dim), len(self.local_fields)
        if self.split_wire() and F_me > 0:
            # [s]: [bc][F_me][D] second-order rows, then pad4(bc) first-order partial sums
            out = torch.empty(self.world * self._block(bc, F_me), device=recv_idx.device, dtype=torch.float32)
            if bc == 0:
                return out
            from ._lib import Segment
            second = [Segment(self.second_order_embeddings[f].weight.data_ptr(), None, 0,
                              self.second_order_embeddings[f].weight.stride(0), self.field_rows[f],
                              self.embedding_dim, 0) for f in self.local_fields]
            first = [Segment(self.first_order_embeddings[f].weight.data_ptr(), None, 0,
                             self.first_order_embeddings[f].weight.stride(0), self.field_rows[f], 1, 0)
                     for f in self.local_fields]
            lib = ops._lib.load()
            ops._lib.ensure_device(out.device)
            ops.check(lib.rk_shard_gather_rows_split(ops._seg_array(second), ops._seg_array(first), F_me,
                                                     self.embedding_dim, recv_idx.data_ptr(), self.world, B_src, b0,
                                                     bc, out.data_ptr(), ops._lib.stream_of(out)),
                      "rk_shard_gather_rows_split")
            return out
        if recv_idx.dtype == torch.int32 and F_me > 0:
            out = torch.empty(self.world * bc, F_me * RS, device=recv_idx.device, dtype=torch.float32)
            if bc == 0:
                return out
            from ._lib import Segment
            segs = [Segment(self.packed_table(f).data_ptr(), None, 0, self.packed_table(f).stride(0),
                            self.packed_table(f).shape[0], RS, 0) for f in self.local_fields]
            lib = ops._lib.load()
            ops._lib.ensure_device(out.device)
            ops.check(lib.rk_shard_gather_rows(ops._seg_array(segs), F_me, RS, recv_idx.data_ptr(), self.world, B_src,
                                               b0, bc, out.data_ptr(), ops._lib.stream_of(out)), "rk_shard_gather_rows")
            return out
        if b0 == 0 and bc == B_src:
            return self.gather_local(recv_idx, self.world * B_src)
        sel = recv_idx.view(self.world, B_src, F_me)[:, b0:b0 + bc].reshape(-1)
        return self.gather_local(sel, self.world * bc)

    def gather_local(self, recv_idx: torch.Tensor, rows_total: int) -> torch.Tensor:
        """Step 2: rows [s*B_l + b][f_me][RS] from this rank's tables (rk_concat_gather)."""
        D, RS, F_me = self.embedding_dim, row_stride(self.embedding_dim), len(self.local_fields)
        out = torch.empty(rows_total, F_me * RS, device=recv_idx.device, dtype=torch.float32)
        if F_me == 0 or rows_total == 0:
            return out
        if recv_idx.dtype != torch.int64:  # int32 wire format
            recv_idx = recv_idx.to(torch.int64)
        segs = []
        for j, f in enumerate(self.local_fields):
            idx = recv_idx[j:]  # element (R, j) sits at R * F_me + j
            segs.append(ops.table_segment(self.packed_table(f), idx, j * RS, idx_stride=F_me))
        ops.concat_gather(segs, rows_total, out)  # whole packed rows, 16-B vectorised path
        return out

    def exchange_rows(self, rows: torch.Tensor, B_l: int, async_op: bool = False):
        """Step 3: send [s][b][f_me][RS] back to every source; receive [r][b][f_r][RS]."""
        out_s, in_s = self.row_splits(B_l)
        recv = torch.empty(sum(out_s), device=rows.device, dtype=torch.float32)
        return self._exchange(recv, rows.reshape(-1), out_s, in_s, async_op)

    def _front_ok(self, B_l: int) -> bool:
        D = self.embedding_dim
        return (self.fused_front and B_l > 0 and len(self._tail) >= 2 and len(self.fields) <= 32
                and 4 <= D <= 256 and D & (D - 1) == 0)

    def _front_and_tail(self, segs, B_l: int):
        """rk_fm_linear_packed (gather, fm1, fm2 and deep layer 0, deepfm.py:122-142 + 100-112)
        then the rest of the tail and the head (deepfm.py:143-151)."""
        from . import common
        dev = self._device()
        widths = [l.linear.out_features for l in self._tail]
        if self.fused_whole and ops.deepfm_whole_plan(len(self.fields) * self.embedding_dim, widths):
            # the whole forward in one rk_deepfm_forward launch (configs[4]: 30 fields x 32, 512-256-128)
            mls = [ops.make_mlp_layer(l.linear.weight, common.PACKED(l.linear.weight), **l.epilogue_kwargs())
                   for l in self._tail]
            fm1, fm2, deep, total, prob = (torch.empty(B_l, 1, device=dev, dtype=torch.float32) for _ in range(5))
            ep = ops.make_epilogue(head_w=self.deep_output_layer.weight, head_b=self.deep_output_layer.bias,
                                   final_w=self.final_layer.weight, final_b=self.final_layer.bias, head_logit=total,
                                   head_prob=prob, head_aux=deep)
            ops.deepfm_forward(segs, self.embedding_dim, B_l, mls, ep, fm1, fm2)
            return prob, total, fm1, fm2, deep
        l0 = self._tail[0]
        ml0 = ops.make_mlp_layer(l0.linear.weight, common.PACKED(l0.linear.weight), **l0.epilogue_kwargs())
        y = torch.empty(B_l, l0.linear.out_features, device=dev, dtype=torch.float32)
        fm1 = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        fm2 = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        ops.fm_linear_packed(segs, self.embedding_dim, B_l, ml0, y, fm1, fm2)
        deep = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        total = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        run_tail(y, self._tail[1:], self.deep_output_layer,
                 dict(fm1=fm1, fm2=fm2, final_w=self.final_layer.weight, final_b=self.final_layer.bias,
                      head_aux=deep), total, prob)
        return prob, total, fm1, fm2, deep

    def fm_and_tail(self, recv_rows: torch.Tensor, B_l: int):
        """Step 4: FM + deep tail on the received rows (field order restored by out_col)."""
        D, RS = self.embedding_dim, row_stride(self.embedding_dim)
        dev = recv_rows.device
        if self.split_wire():
            # owner r's block: [B_l][F_r][D] rows then pad4(B_l) first-order partials; the partials
            # ride on the owner's first field (the others contribute no first-order term)
            from ._lib import Segment
            segs, first, first_ld = [], [], []
            off, place = 0, {}
            for r in range(self.world):
                F_r = len(self.fields_of[r])
                for j, f in enumerate(self.fields_of[r]):
                    place[f] = (off + j * D, F_r * D, off + B_l * F_r * D if j == 0 else None)
                off += self._block(B_l, F_r)
            base = recv_rows.data_ptr()
            for i, f in enumerate(self.fields):
                o, ld, po = place[f]
                segs.append(Segment(base + 4 * o, None, 0, ld, 0, D, i * D))
                first.append(base + 4 * po if po is not None else None)
                first_ld.append(1 if po is not None else 0)
            mls = [ops.make_mlp_layer(l.linear.weight, common_packed(l.linear.weight), **l.epilogue_kwargs())
                   for l in self._tail]
            fm1, fm2, deep, total, prob = (torch.empty(B_l, 1, device=dev, dtype=torch.float32) for _ in range(5))
            ep = ops.make_epilogue(head_w=self.deep_output_layer.weight, head_b=self.deep_output_layer.bias,
                                   final_w=self.final_layer.weight, final_b=self.final_layer.bias, head_logit=total,
                                   head_prob=prob, head_aux=deep)
            if B_l > 0:
                ops.deepfm_forward_fo(segs, first, first_ld, D, B_l, mls, ep, fm1, fm2)
            return prob, total, fm1, fm2, deep
        second, first = [], []
        off = 0
        base = {}
        for r in range(self.world):
            for j, f in enumerate(self.fields_of[r]):
                base[f] = (off + j * RS, len(self.fields_of[r]) * RS)
            off += B_l * len(self.fields_of[r]) * RS
        if self._front_ok(B_l):  # the received packed rows read in place (dense segments)
            from ._lib import Segment
            segs = [Segment(recv_rows.data_ptr() + base[f][0] * 4, None, 0, base[f][1], 0, D, i * D)
                    for i, f in enumerate(self.fields)]
            return self._front_and_tail(segs, B_l)
        for i, f in enumerate(self.fields):
            o, ld = base[f]
            second.append(_lib_dense(recv_rows, o, ld, D, i * D))
            first.append(_lib_dense(recv_rows, o + D, ld, 1, i))
        deep_in = torch.empty(B_l, len(self.fields) * D, device=dev, dtype=torch.float32)
        fm1 = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        fm2 = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        ops.fm_gather(second, first, D, B_l, deep_in, fm1, fm2)
        return self._tail_of(deep_in, fm1, fm2)

    def local_fm_and_tail(self, cat: dict):
        """P = 1: the FM gather straight from the packed tables (one pass), then the tail."""
        D = self.embedding_dim
        B_l = cat[self.fields[0]].shape[0]
        dev = self._device()
        segs = []
        for i, f in enumerate(self.fields):
            idx = cat[f] if cat[f].stride(0) == 1 else cat[f].contiguous()
            segs.append(ops.packed_segment(self.packed_table(f), idx, D, i * D))
        if self._front_ok(B_l):
            return self._front_and_tail(segs, B_l)
        deep_in = torch.empty(B_l, len(self.fields) * D, device=dev, dtype=torch.float32)
        fm1 = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        fm2 = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        ops.fm_gather_packed(segs, D, B_l, deep_in, fm1, fm2)
        return self._tail_of(deep_in, fm1, fm2)

    def _tail_of(self, deep_in, fm1, fm2):
        B_l, dev = deep_in.shape[0], deep_in.device
        deep = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        total = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B_l, 1, device=dev, dtype=torch.float32)
        run_tail(deep_in, self._tail, self.deep_output_layer,
                 dict(fm1=fm1, fm2=fm2, final_w=self.final_layer.weight, final_b=self.final_layer.bias,
                      head_aux=deep), total, prob)
        return prob, total, fm1, fm2, deep

    def _device(self):
        return self.deep_output_layer.weight.device

    def forward(self, category: dict):
        """category: {field: [B_l] int64} for every field, this rank's samples."""
        check_eval(self)
        missing = [f for f in self.fields if f not in category]
        if missing:
            raise KeyError(f"ShardedDeepFM.forward: category features missing: {missing}")
        cat = {f: ops.as_index(category[f], f"category[{f!r}]") for f in self.fields}
        return self.run_steps(cat)

    def chunk_bounds(self, B_l: int, chunks: int = None):
        """Sample ranges of the exchange pipeline (overlap the row all-to-all with
        compute): `pipeline_chunks` contiguous slices of the local batch, none under `min_chunk` samples."""
        C = self.pipeline_chunks if chunks is None else chunks
        C = max(1, min(C, B_l // self.min_chunk))
        edges = [B_l * i // C for i in range(C + 1)]
        return [(edges[i], edges[i + 1]) for i in range(C)]

    def run_steps(self, cat: dict, chunks: int = None):
        """P > 1: one index all-to-all for the whole local batch, then steps 2-4 per chunk,
        pipelined — each chunk's gather runs on the compute stream while the previous chunk's row
        all-to-all is in flight on the collective stream; the FM + tail of a chunk waits only for
        its own rows.  Outputs are the chunks' results in sample order (each sample's math is
        independent of the chunking)."""
        if self.world == 1:
            return self.local_fm_and_tail(cat)
        B_l = cat[self.fields[0]].shape[0]
        parts = self.chunk_bounds(B_l, chunks)
        recv_idx, work = self.exchange_indices(cat, B_l, async_op=True)
        if work is not None:
            work.wait()
        rows = []
        for b0, b1 in parts:
            rows.append(self.exchange_rows(self.gather_rows(recv_idx, B_l, b0, b1 - b0), b1 - b0, async_op=True))
        outs = []
        for (recv_rows, work), (b0, b1) in zip(rows, parts):
            if work is not None:
                work.wait()
            outs.append(self.fm_and_tail(recv_rows, b1 - b0))
        if len(outs) == 1:
            return outs[0]
        return tuple(torch.cat([o[i] for o in outs], 0) for i in range(len(outs[0])))

    def pipeline(self, batch: int, *, side_stream: bool = True, capture=None) -> "ExchangePipeline":
        """The cross-batch exchange pipeline (P > 1) for local batches of `batch` samples: push()
        batch i, get back batch i - 2's outputs; the exchanges of the two younger batches run under
        the older one's forward (ExchangePipeline).  capture=[3 device batches]: the local segments
        as hipGraphs bound to those batches (bench.py)."""
        return ExchangePipeline(self, batch, side_stream=side_stream, capture=capture)

    def capture_pipeline(self, cat: dict, chunks: int = None) -> "CapturedPipeline":
        """run_steps with each chunk's three local segments (index pack, gather, FM + tail)
        captured as hipGraphs; the all-to-alls stay outside the graphs (RCCL collectives are
        issued per step with async_op, so chunk c's rows travel while chunk c+1 gathers).
        Capture is local (no collective), so the ranks may capture in any order."""
        return CapturedPipeline(self, cat, chunks)


def _graph_of(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.no_grad():
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    # thread_local: RCCL's watchdog thread queries its events during the capture (only this
    # thread's calls are restricted)
    with torch.no_grad(), torch.cuda.graph(g, capture_error_mode="thread_local"):
        out = fn()
    return g, out


class CapturedPipeline:
    """The P > 1 exchange pipeline of ShardedDeepFM.run_steps as replayable segments.  step()
    issues: pack graph -> index all-to-all (whole local batch) -> per chunk: gather graph -> async
    row all-to-all; then per chunk: wait -> FM + tail graph.  `outputs` are the five forward outputs
    of the last step (concatenated over chunks by result())."""

    def __init__(self, model: ShardedDeepFM, cat: dict, chunks: int = None):
        if model.world == 1:
            raise ValueError("capture_pipeline: P = 1 has no exchange; capture run_steps as one graph")
        self.model = model
        dev = model._device()
        B_l = cat[model.fields[0]].shape[0]
        out_i, in_i = model.index_splits(B_l)
        self.idx_splits = (out_i, in_i)
        self.recv_idx = torch.zeros(sum(out_i), dtype=model.index_dtype, device=dev)  # valid rows for the warm-ups
        self.g_pack, self.send = _graph_of(lambda: model.pack_indices(cat))
        self.segs = []
        for b0, b1 in model.chunk_bounds(B_l, chunks):
            Bc = b1 - b0
            out_r, in_r = model.row_splits(Bc)
            recv_rows = torch.empty(sum(out_r), dtype=torch.float32, device=dev)
            g2, rows = _graph_of(lambda b0=b0, Bc=Bc: model.gather_rows(self.recv_idx, B_l, b0, Bc))
            g3, outs = _graph_of(lambda rr=recv_rows, Bc=Bc: model.fm_and_tail(rr, Bc))
            self.segs.append(dict(g2=g2, rows=rows, g3=g3, outs=outs, recv_rows=recv_rows, row_splits=(out_r, in_r)))

    def step(self):
        m = self.model
        self.g_pack.replay()
        w = m._exchange(self.recv_idx, self.send, *self.idx_splits, async_op=True)[1]
        if w is not None:
            w.wait()
        rworks = []
        for s in self.segs:
            s["g2"].replay()
            rworks.append(m._exchange(s["recv_rows"], s["rows"].reshape(-1), *s["row_splits"], async_op=True)[1])
        for s, w in zip(self.segs, rworks):
            if w is not None:
                w.wait()
            s["g3"].replay()

    def result(self):
        outs = [s["outs"] for s in self.segs]
        if len(outs) == 1:
            return outs[0]
        return tuple(torch.cat([o[i] for o in outs], 0) for i in range(len(outs[0])))


def common_packed(w):
    from . import common
    return common.PACKED(w)


def _lib_dense(buf: torch.Tensor, offset: int, ld: int, dim: int, out_col: int):
    from ._lib import Segment
    return Segment(buf.data_ptr() + offset * 4, None, 0, ld, 0, dim, out_col)


class _Ring:
    """One pipeline slot's device buffers (index send/receive, row send/receive)."""

    def __init__(self, model: "ShardedDeepFM", B_l: int, dev):
        out_i, in_i = model.index_splits(B_l)
        out_r, in_r = model.row_splits(B_l)
        self.send_idx = torch.zeros(sum(in_i), dtype=model.index_dtype, device=dev)
        self.recv_idx = torch.zeros(sum(out_i), dtype=model.index_dtype, device=dev)
        self.recv_rows = torch.zeros(sum(out_r), dtype=torch.float32, device=dev)
        self.send_rows = None  # gather output (allocated by the gather; captured: fixed)
        self.idx_work = self.row_work = None
        self.fwd_done = None  # event after the forward that last read recv_rows


class ExchangePipeline:
    """ShardedDeepFM's P > 1 step as a cross-batch software pipeline.

    Batch i moves through three stages on three consecutive push() calls:

      A(i)    pack(i)   -> index all_to_all_single(i), async          [side stream]
      B(i)    wait index(i) -> gather_rows(i) -> row all_to_all(i), async  [side stream]
      C(i)    wait rows(i)  -> the one-launch forward over the received rows [compute stream]

    push(batch i) issues B(i-1), A(i), C(i-2) and returns batch i-2's outputs, so the index and row
    exchanges of the two younger batches are in flight (RCCL on the process group's stream) while
    the oldest one's forward runs: a step costs max(local device work, wire) instead of their sum,
    and the forward covers the whole local batch in one rk_deepfm_forward launch (32-row workgroups
    from 8,192 rows) — no chunking.  Three buffer slots rotate (batch i uses slot i % 3); every reuse
    is stream-ordered behind the last reader of the slot:
      send_idx   rewritten by pack(i+3) on the side stream, which waited for index(i) at B(i);
      recv_idx   rewritten by index(i+3), issued from the side stream after B(i)'s gather;
      send rows  rewritten by gather(i+3), which waits for index(i+3), queued behind row(i)
                 on the collective stream (one stream per process group);
      recv_rows  rewritten by row(i+3), issued after the side stream waited for C(i)'s event.
    Collectives are issued in the same order on every rank (B(i-1)'s rows, then A(i)'s indices).
    flush() drains the two batches still in flight.  Every sample's arithmetic is that of
    ShardedDeepFM.run_steps: outputs are identical to the unpipelined forward.

    CPU tensors (gloo): no streams; async work handles are waited on the host."""

    DEPTH = 3

    def __init__(self, model: "ShardedDeepFM", batch: int, *, side_stream: bool = True, capture=None):
        if model.world == 1:
            raise ValueError("ExchangePipeline: P = 1 has no exchange (use the model's forward)")
        check_eval(model)
        self.model, self.B = model, int(batch)
        dev = model._device()
        self.cuda = dev.type == "cuda"
        self.main = torch.cuda.current_stream(dev) if self.cuda else None
        self.side = (torch.cuda.Stream(dev) if side_stream else self.main) if self.cuda else None
        self.slots = [_Ring(model, self.B, dev) for _ in range(self.DEPTH)]
        self.n_in = 0    # batches pushed
        self.n_out = 0   # batches whose forward has been issued
        self.cats = [None] * self.DEPTH
        self.graphs = None
        if capture is not None:
            self._capture(capture)

    def _capture(self, cats):
        """Captured mode (bench.py's P > 1 step): slot k's pack (bound to the index tensors cats[k]),
        gather and forward as three hipGraphs, replayed by the stages on the same streams; the
        collectives stay outside the graphs.  push() then takes the slot's bound batch (its
        contents may change between pushes) and returns the slot's fixed output tensors, valid
        until the slot's next forward (three pushes later)."""
        if not self.cuda or len(cats) != self.DEPTH:
            raise ValueError(f"ExchangePipeline capture: {self.DEPTH} device batches needed")
        m = self.model
        graphs = []
        for k, cat in enumerate(cats):
            cat = {f: ops.as_index(cat[f], f"category[{f!r}]") for f in m.fields}
            sl = self.slots[k]
            g_pack, sl.send_idx = _graph_of(lambda c=cat: m.pack_indices(c))
            g_gather, sl.send_rows = _graph_of(lambda sl=sl: m.gather_rows(sl.recv_idx, self.B, 0, self.B))
            g_fwd, outs = _graph_of(lambda sl=sl: m.fm_and_tail(sl.recv_rows, self.B))
            graphs.append({"pack": g_pack, "gather": g_gather, "forward": g_fwd, "outs": outs, "cat": cat})
            self.cats[k] = cat
        self.graphs = graphs

    def step(self):
        """Captured mode: one pipeline step on the slots' bound batches (push without the checks)."""
        i = self.n_in
        if i >= 1:
            self._stage_b(i - 1)
        self._stage_a(i, None)
        self.n_in += 1
        if i >= 2:
            self.n_out += 1
            return self._stage_c(i - 2)
        return None

    # -- stream helpers
    def _on(self, st):
        import contextlib
        return torch.cuda.stream(st) if self.cuda else contextlib.nullcontext()

    @staticmethod
    def _wait(work):
        if work is not None:
            work.wait()  # stream-ordered on CUDA (the current stream waits), host-blocking on gloo

    # -- stages
    def _stage_a(self, i: int, cat: dict):
        m, sl = self.model, self.slots[i % self.DEPTH]
        if self.cuda and self.side is not self.main:
            self.side.wait_stream(self.main)  # the caller's index tensors were written on the compute stream
        with self._on(self.side):
            if self.graphs:
                self.graphs[i % self.DEPTH]["pack"].replay()
                send = sl.send_idx
            else:
                send = sl.send_idx = m.pack_indices(cat)
            out_s, in_s = m.index_splits(self.B)
            sl.idx_work = m._exchange(sl.recv_idx, send, out_s, in_s, async_op=True)[1]

    def _stage_b(self, i: int):
        m, sl = self.model, self.slots[i % self.DEPTH]
        with self._on(self.side):
            self._wait(sl.idx_work)
            sl.idx_work = None
            if self.graphs:
                self.graphs[i % self.DEPTH]["gather"].replay()
            else:
                sl.send_rows = m.gather_rows(sl.recv_idx, self.B, 0, self.B)
            if sl.fwd_done is not None:  # C(i-3) read recv_rows: the row exchange may overwrite it now
                self.side.wait_event(sl.fwd_done)
            out_s, in_s = m.row_splits(self.B)
            sl.row_work = m._exchange(sl.recv_rows, sl.send_rows.reshape(-1), out_s, in_s, async_op=True)[1]

    def _stage_c(self, i: int):
        m, sl = self.model, self.slots[i % self.DEPTH]
        with self._on(self.main):
            self._wait(sl.row_work)
            sl.row_work = None
            if self.graphs:
                self.graphs[i % self.DEPTH]["forward"].replay()
                out = self.graphs[i % self.DEPTH]["outs"]
            else:
                out = m.fm_and_tail(sl.recv_rows, self.B)
            if self.cuda:
                sl.fwd_done = torch.cuda.Event()
                sl.fwd_done.record(self.main)
        return out

    # -- driver
    def push(self, category: dict):
        """Feed one local batch ({field: [batch] int64}); returns the outputs (prob, total_logit,
        fm1, fm2, deep_logit) of the batch pushed two calls earlier, or None while the pipeline fills."""
        m = self.model
        if self.graphs:
            return self.step()
        missing = [f for f in m.fields if f not in category]
        if missing:
            raise KeyError(f"ExchangePipeline.push: category features missing: {missing}")
        # (device checks on the GPU path; the gloo tests drive CPU stand-ins of the device steps)
        cat = ({f: ops.as_index(category[f], f"category[{f!r}]") for f in m.fields} if self.cuda
               else {f: category[f] for f in m.fields})
        if cat[m.fields[0]].shape[0] != self.B:
            raise ValueError(f"ExchangePipeline.push: batch {cat[m.fields[0]].shape[0]} != {self.B}")
        i = self.n_in
        if i >= 1:
            self._stage_b(i - 1)
        self._stage_a(i, cat)
        self.cats[i % self.DEPTH] = cat  # the index tensors stay alive until pack(i) has read them
        self.n_in += 1
        if i >= 2:
            self.n_out += 1
            return self._stage_c(i - 2)
        return None

    def flush(self):
        """Outputs of the batches still in flight, oldest first (the pipeline is empty afterwards)."""
        outs = []
        i = self.n_in
        # C of the older batch in flight, B of the newest (its A ran in the last push), then its C
        if i >= 2 and self.n_out == i - 2:
            outs.append(self._stage_c(i - 2))
            self.n_out += 1
        if i >= 1:
            self._stage_b(i - 1)
        while self.n_out < i:
            outs.append(self._stage_c(self.n_out))
            self.n_out += 1
        self.n_in = self.n_out = 0
        if not self.graphs:
            for sl in self.slots:
                sl.send_rows = None
        return outs
