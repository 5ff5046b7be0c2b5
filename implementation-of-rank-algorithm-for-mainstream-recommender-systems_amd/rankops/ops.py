"""Thin Python wrappers over the rankops C ABI.

Each wrapper validates devices/dtypes/shapes, turns tensors into device pointers and launches
on the current HIP stream of the tensors' device.  Outputs are allocated from PyTorch's
caching allocator, so every wrapper is safe inside `torch.cuda.graph` capture.  There is no
CPU path: a CPU tensor is an error (the CPU restatement in oracle/ is test-only).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from ._lib import Epilogue, Segment, check, fptr, ptr

ACT = {"none": _lib.RK_ACT_NONE, "relu": _lib.RK_ACT_RELU, "leaky": _lib.RK_ACT_LEAKY,
       "dice": _lib.RK_ACT_DICE, "prelu": _lib.RK_ACT_PRELU}


def require_gpu(t: torch.Tensor, what: str):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"rankops: {what} must be a tensor, got {type(t).__name__}")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"rankops: {what} is on {t.device}; the rankops forward runs only on a ROCm GPU "
            f"(move the model and inputs with .to('cuda'))")
    return t


def as_index(t: torch.Tensor, what: str) -> torch.Tensor:
    require_gpu(t, what)
    if t.dtype != torch.int64:
        if t.dtype in (torch.int32, torch.int16, torch.uint8, torch.int8):
            t = t.long()
        else:
            raise TypeError(f"rankops: {what} must be an integer tensor, got {t.dtype}")
    return t


def bound_index(t: torch.Tensor, what: str, contiguous: bool = False) -> torch.Tensor:
    """An index tensor a prepared launch binds by address (Model.prepare): it must be the caller's
    own int64 tensor (and contiguous where the kernel reads it as a dense block), since a converted
    copy would silently stop following later writes to the caller's tensor."""
    require_gpu(t, what)
    if t.dtype != torch.int64:
        raise TypeError(f"rankops: prepare() binds {what} by address; it must be int64 (got {t.dtype}): "
                        "convert it once and pass the converted tensor")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"rankops: prepare() binds {what} by address; it must be contiguous")
    return t


def as_f32(t: torch.Tensor, what: str) -> torch.Tensor:
    require_gpu(t, what)
    if t.dtype != torch.float32:
        raise TypeError(f"rankops: {what} must be float32, got {t.dtype}")
    return t


def table_segment(weight: torch.Tensor, idx: torch.Tensor, out_col: int, idx_stride: int = None) -> Segment:
    """Embedding-table segment: rows weight[idx[b]] -> out[b, out_col:out_col+dim]."""
    if weight.dim() != 2 or weight.stride(1) != 1:
        raise ValueError("rankops: embedding weight must be 2-D with unit column stride")
    if idx_stride is None:
        if idx.dim() != 1:
            raise ValueError(f"rankops: expected a 1-D index tensor, got shape {tuple(idx.shape)}")
        idx_stride = idx.stride(0)
    return Segment(weight.data_ptr(), idx.data_ptr(), idx_stride, weight.stride(0), weight.shape[0],
                   weight.shape[1], out_col)


def packed_segment(packed: torch.Tensor, idx: torch.Tensor, dim: int, out_col: int) -> Segment:
    """Packed FM-table segment (rk_fm_gather_packed): row packed[idx[b]], D floats + weight at D."""
    if idx.dim() != 1 or idx.stride(0) != 1:
        raise ValueError("rankops: packed FM gather needs unit-stride 1-D indices")
    return Segment(packed.data_ptr(), idx.data_ptr(), 1, packed.stride(0), packed.shape[0], dim, out_col)


def dense_segment(src: torch.Tensor, dim: int, out_col: int, col_offset: int = 0) -> Segment:
    """Dense segment: src[b, col_offset:col_offset+dim] -> out[b, out_col:+dim] (src is [B] or [B, *])."""
    if src.dim() == 1:
        if dim != 1:
            raise ValueError("rankops: a 1-D dense source has dim 1")
        ld = src.stride(0)
    else:
        if src.stride(-1) != 1:
            raise ValueError("rankops: dense source must have unit column stride")
        ld = src.stride(0)
    return Segment(fptr(src, col_offset), None, 0, ld, 0, dim, out_col)


def _seg_array(segs):
    arr = (Segment * len(segs))(*segs)
    return arr


_SEG_ARRAYS = {}


def table_seg_array(weights, idxs, cols):
    """The rk_segment array of table segments weights[k][idxs[k]] -> column cols[k], memoized on
    every field of the structs (pointers, strides, shapes): a repeated training step, whose tables,
    index tensors and (recycled) gradient buffers come back at the same addresses, reuses the
    marshalled array instead of building a ctypes struct per field.  The library copies the array
    into the kernel arguments at launch, so sharing it is safe."""
    key = tuple((w.data_ptr(), w.stride(0), w.shape[0], w.shape[1], w.stride(1), i.data_ptr(), i.stride(0), i.dim(), c)
                for w, i, c in zip(weights, idxs, cols))
    arr = _SEG_ARRAYS.get(key)
    if arr is None:
        arr = _seg_array([table_segment(w, i, c) for w, i, c in zip(weights, idxs, cols)])
        if len(_SEG_ARRAYS) >= 512:
            _SEG_ARRAYS.clear()
        _SEG_ARRAYS[key] = arr
    return arr


def dense_table_seg_array(dense, ndense, weights, idxs):
    """[dense columns 0..ndense) + table segments side by side] as a memoized rk_segment array
    (DCN / DeepCrossing feature rows; table_seg_array's rules)."""
    key = (dense.data_ptr(), dense.stride(0), dense.dim(), ndense) + tuple(
        (w.data_ptr(), w.stride(0), w.shape[0], w.shape[1], w.stride(1), i.data_ptr(), i.stride(0), i.dim())
        for w, i in zip(weights, idxs))
    arr = _SEG_ARRAYS.get(key)
    if arr is None:
        segs, col = [dense_segment(dense, ndense, 0)], ndense
        for w, i in zip(weights, idxs):
            segs.append(table_segment(w, i, col))
            col += w.shape[1]
        arr = _seg_array(segs)
        if len(_SEG_ARRAYS) >= 512:
            _SEG_ARRAYS.clear()
        _SEG_ARRAYS[key] = arr
    return arr


def concat_gather(segs, batch: int, out: torch.Tensor):
    lib = _lib.load()
    _lib.ensure_device(out.device)
    arr = _seg_array(segs)
    check(lib.rk_concat_gather(arr, len(segs), batch, ptr(out), out.stride(0), _lib.stream_of(out)),
          "rk_concat_gather")
    return out


def dcn_cross(segs, batch, width, cross_w, cross_b, num_layers, head_w_ptr, x0, partial, device,
              xl_in=None, xl_out=None):
    lib = _lib.load()
    _lib.ensure_device(device)
    arr = _as_seg_array(segs)
    check(lib.rk_dcn_cross(arr, len(segs), batch, width, ptr(cross_w), ptr(cross_b), num_layers, head_w_ptr,
                           ptr(x0), x0.stride(0) if x0 is not None else 0,
                           ptr(xl_in), xl_in.stride(0) if xl_in is not None else 0,
                           ptr(xl_out), xl_out.stride(0) if xl_out is not None else 0,
                           ptr(partial), _lib.raw_stream(device)), "rk_dcn_cross")


def dcn_forward_args(segs, batch, width, cross_w, cross_b, num_layers, cross_head_w, layers, head: Epilogue,
                     device):
    """The rk_dcn_forward argument list (the stream last, None) — cross_w / cross_b at [4] / [5] and
    the stream at [-1] are the per-call slots of a cached eager forward (DCNModel)."""
    _lib.ensure_device(device)
    arr = _seg_array(segs)
    mls = (_lib.MlpLayer * max(1, len(layers)))(*layers)
    return [arr, len(segs), batch, width, ptr(cross_w), ptr(cross_b), num_layers, cross_head_w.data_ptr(), mls,
            len(layers), ctypes.byref(head), None]


def dcn_forward(segs, batch, width, cross_w, cross_b, num_layers, cross_head_w, layers, head: Epilogue,
                device):
    """rk_dcn_forward: gather + cross stack + MLP tail + head in one launch (DCNModel eval forward)."""
    args = dcn_forward_args(segs, batch, width, cross_w, cross_b, num_layers, cross_head_w, layers, head, device)
    args[-1] = _lib.raw_stream(device)
    check(_lib.load().rk_dcn_forward(*args), "rk_dcn_forward")


def fm_gather(second, first, dim, batch, deep_in, fm1, fm2):
    lib = _lib.load()
    _lib.ensure_device(deep_in.device)
    a2, a1 = _as_seg_array(second), _as_seg_array(first)
    check(lib.rk_fm_gather(a2, a1, len(second), dim, batch, ptr(deep_in), deep_in.stride(0), ptr(fm1), ptr(fm2),
                           _lib.stream_of(deep_in)), "rk_fm_gather")


def fm_pack_table(second: torch.Tensor, first: torch.Tensor, row_stride: int) -> torch.Tensor:
    """rk_fm_pack_table: [V, D] + [V, 1] -> one [V, row_stride] table (row, then the weight at D)."""
    lib = _lib.load()
    _lib.ensure_device(second.device)
    V, D = second.shape
    if first.shape[0] != V or second.stride(1) != 1:
        raise ValueError("rankops.fm_pack_table: tables of one field must have the same rows")
    out = torch.empty(V, row_stride, device=second.device, dtype=torch.float32)
    check(lib.rk_fm_pack_table(ptr(second), second.stride(0), ptr(first), first.stride(0), V, D, ptr(out),
                               row_stride, _lib.stream_of(out)), "rk_fm_pack_table")
    return out


def fm_gather_packed(fields, dim, batch, deep_in, fm1, fm2):
    """rk_fm_gather_packed: fields = table_segment(packed table, idx, out_col) per field."""
    lib = _lib.load()
    _lib.ensure_device(deep_in.device)
    arr = _seg_array(fields)
    check(lib.rk_fm_gather_packed(arr, len(fields), dim, batch, ptr(deep_in), deep_in.stride(0), ptr(fm1),
                                  ptr(fm2), _lib.stream_of(deep_in)), "rk_fm_gather_packed")


def fm_linear_packed(fields, dim, batch, layer: "_lib.MlpLayer", y, fm1, fm2):
    """rk_fm_linear_packed: the packed FM gather, fm1, fm2 and the first deep layer into y [batch, n]
    in one launch; fields = packed_segment(table, idx, dim, f * dim) per field."""
    lib = _lib.load()
    _lib.ensure_device(y.device)
    arr = _seg_array(fields)
    check(lib.rk_fm_linear_packed(arr, len(fields), dim, batch, ctypes.byref(layer), ptr(y), y.stride(0), ptr(fm1),
                                  ptr(fm2), _lib.stream_of(y)), "rk_fm_linear_packed")


def deepfm_whole_plan(k0: int, widths) -> bool:
    """Whether rk_deepfm_forward has a compiled plan for this DeepFM (deep input k0 wide, hidden
    widths): 960 -> 512 -> 256 -> 128 (configs[1]); RANKOPS_MLP_STREAM=0 turns it off, as in C."""
    return (os.environ.get("RANKOPS_MLP_STREAM", "1")[:1] != "0" and (k0 + 63) // 64 * 64 == 960
            and list(widths) == [512, 256, 128])


def deepfm_forward(fields, dim, batch, layers, ep, fm1, fm2):
    """rk_deepfm_forward: the whole DeepFM eval forward in one launch (packed gather, FM, the deep
    layers and the head); fields = packed_segment(table, idx, dim, f * dim) per field, layers the
    three MlpLayer structs, ep the head epilogue (head_w/b, final_w/b, head_logit/prob/aux)."""
    lib = _lib.load()
    _lib.ensure_device(fm1.device)
    arr = _seg_array(fields)
    la = (_lib.MlpLayer * len(layers))(*layers)
    check(lib.rk_deepfm_forward(arr, len(fields), dim, batch, la, len(layers), ctypes.byref(ep), ptr(fm1), ptr(fm2),
                                _lib.stream_of(fm1)), "rk_deepfm_forward")


def deepfm_forward_fo(fields, first, first_ld, dim, batch, layers, ep, fm1, fm2):
    """rk_deepfm_forward_fo: rk_deepfm_forward with the first-order weights from their own sources
    (first[f]: a device address or None, first_ld[f] its row stride in floats)."""
    lib = _lib.load()
    _lib.ensure_device(fm1.device)
    arr = _seg_array(fields)
    n = len(fields)
    fp = (ctypes.c_void_p * n)(*[x or None for x in first])
    fl = (ctypes.c_int64 * n)(*first_ld)
    la = (_lib.MlpLayer * len(layers))(*layers)
    check(lib.rk_deepfm_forward_fo(arr, fp, fl, n, dim, batch, la, len(layers), ctypes.byref(ep), ptr(fm1), ptr(fm2),
                                   _lib.stream_of(fm1)), "rk_deepfm_forward_fo")


def din_attention(query_ptr, ld_query, key_table, seq, seq_len, T, H, weights, use_softmax, out_ptr, ld_out,
                  batch, device):
    lib = _lib.load()
    _lib.ensure_device(device)
    w1, b1, w2, b2, w3, b3 = weights
    check(lib.rk_din_attention(query_ptr, ld_query, ptr(key_table), key_table.shape[0], key_table.stride(0),
                               ptr(seq), seq.stride(0), T, ptr(seq_len), batch, H, ptr(w1), ptr(b1), ptr(w2),
                               ptr(b2), ptr(w3), ptr(b3), 1 if use_softmax else 0, out_ptr, ld_out,
                               _lib.raw_stream(device)), "rk_din_attention")


def din_attention_dense(query, keys, keys_length, weights, use_softmax, out):
    """rk_din_attention_dense: keys [B, T, H] (rows 16-B aligned), query/out [B, H]."""
    lib = _lib.load()
    _lib.ensure_device(keys.device)
    w1, b1, w2, b2, w3, b3 = weights
    B, T, H = keys.shape
    check(lib.rk_din_attention_dense(ptr(query), query.stride(0), ptr(keys), keys.stride(0), keys.stride(1), T,
                                     ptr(keys_length), B, H, ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(w3), ptr(b3),
                                     1 if use_softmax else 0, ptr(out), out.stride(0), _lib.stream_of(keys)),
          "rk_din_attention_dense")


def dice_forward(x, scale, shift, alpha, y):
    lib = _lib.load()
    check(lib.rk_dice_forward(ptr(x), x.stride(0), x.shape[0], x.shape[1], ptr(scale), ptr(shift), ptr(alpha),
                              ptr(y), y.stride(0), _lib.stream_of(x)), "rk_dice_forward")


L2_WORKSPACE = 512  # RK_L2_WORKSPACE


def row_l2norm_mean(x: torch.Tensor, col0: int, ncols: int, scale: float, out: torch.Tensor):
    lib = _lib.load()
    ws = torch.empty(L2_WORKSPACE, device=x.device, dtype=torch.float32)
    check(lib.rk_row_l2norm_mean(ptr(x), x.stride(0), x.shape[0], col0, ncols, scale, ptr(ws), ptr(out),
                                 _lib.stream_of(x)), "rk_row_l2norm_mean")
    return out


def afm_forward_args(fields, dim, batch, dense, dense_w, dense_b, att_w, att_b, att_h, att_hb, p_w, p_b, logit, prob):
    """The argument tuple of one rk_afm_forward call (the segment array is part of it)."""
    _lib.ensure_device(logit.device)
    arr = _seg_array(fields)
    nd = dense.shape[1] if dense is not None else 0
    return (arr, len(fields), dim, batch, ptr(dense), dense.stride(0) if dense is not None else 0, nd, ptr(dense_w),
            ptr(dense_b), ptr(att_w), ptr(att_b), att_w.shape[0], ptr(att_h), ptr(att_hb), ptr(p_w), ptr(p_b),
            ptr(logit), ptr(prob), _lib.stream_of(logit))


def afm_forward(fields, dim, batch, dense, dense_w, dense_b, att_w, att_b, att_h, att_hb, p_w, p_b, logit, prob):
    check(_lib.load().rk_afm_forward(*afm_forward_args(fields, dim, batch, dense, dense_w, dense_b, att_w, att_b, att_h,
                                                       att_hb, p_w, p_b, logit, prob)), "rk_afm_forward")


def _as_seg_array(segs):
    return segs if isinstance(segs, ctypes.Array) else _seg_array(segs)


def fwfm_forward(emb, lin, dim, batch, field_weight, bias, logit, prob):
    """emb / lin: lists of Segments or ready rk_segment arrays (table_seg_array)."""
    lib = _lib.load()
    _lib.ensure_device(prob.device)
    check(lib.rk_fwfm_forward(_as_seg_array(emb), _as_seg_array(lin), len(emb), dim, batch, ptr(field_weight),
                              ptr(bias), ptr(logit), ptr(prob), _lib.stream_of(prob)), "rk_fwfm_forward")


def bst_attention(qkv, batch, T, d_model, heads, seq_len, ctx):
    lib = _lib.load()
    check(lib.rk_bst_attention(ptr(qkv), qkv.stride(0), batch, T, d_model, heads, ptr(seq_len), ptr(ctx),
                               ctx.stride(0), _lib.stream_of(qkv)), "rk_bst_attention")


def bst_attention_masked(qkv, batch, T, d_model, heads, key_mask, ctx):
    """key_mask: None or a [batch, T] uint8 view of the bool key_padding_mask (nonzero = masked)."""
    lib = _lib.load()
    check(lib.rk_bst_attention_masked(ptr(qkv), qkv.stride(0), batch, T, d_model, heads, ptr(key_mask),
                                      key_mask.stride(0) if key_mask is not None else 0, ptr(ctx), ctx.stride(0),
                                      _lib.stream_of(qkv)), "rk_bst_attention_masked")


BST_BLOCK_PARAMS = 17


def bst_forward_blocks(table, seq, seq_len, d_model, heads, blocks, pool_out_ptr, ld_pool, pool_mean,
                       packed=False):
    """rk_bst_forward_blocks: `blocks` = list of (17 device tensors in the header's order,
    (ln1_eps, ln2_eps, slope)); packed: the six projection weights in rk_bst_pack_block_weight's
    layout (rk_bst_forward_blocks_packed)."""
    lib = _lib.load()
    fn, name = ((lib.rk_bst_forward_blocks_packed, "rk_bst_forward_blocks_packed") if packed else
                (lib.rk_bst_forward_blocks, "rk_bst_forward_blocks"))
    B, T = seq.shape
    params = (ctypes.c_void_p * (BST_BLOCK_PARAMS * len(blocks)))()
    scalars = (ctypes.c_float * (3 * len(blocks)))()
    for i, (tensors, sc) in enumerate(blocks):
        assert len(tensors) == BST_BLOCK_PARAMS
        for k, t in enumerate(tensors):
            params[BST_BLOCK_PARAMS * i + k] = ptr(t)
        for k in range(3):
            scalars[3 * i + k] = float(sc[k])
    check(fn(ptr(table), table.shape[0], table.stride(0), ptr(seq), seq.stride(0), T, ptr(seq_len), B, d_model, heads,
             len(blocks), params, scalars, pool_out_ptr, ld_pool, 1 if pool_mean else 0, _lib.stream_of(table)), name)


def pack_bst_weight(weight: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """[128, 128] BST projection weight -> rk_bst_pack_block_weight's MFMA load order (into `out`
    when given: a previous image, rewritten in place)."""
    lib = _lib.load()
    require_gpu(weight, "bst weight")
    if tuple(weight.shape) != (128, 128) or weight.dtype != torch.float32:
        raise ValueError(f"pack_bst_weight: expected a float32 [128, 128] weight, got {tuple(weight.shape)}")
    w = weight.detach().contiguous()
    if out is None:
        out = torch.empty(128, 128, device=w.device, dtype=torch.float32)
    check(lib.rk_bst_pack_block_weight(w.data_ptr(), out.data_ptr(), _lib.stream_of(out)), "rk_bst_pack_block_weight")
    return out


def bst_small_forward_args(segs, width, table, seq, seq_len, heads, blocks, pool_mean, layers, head: Epilogue):
    """The argument tuple of one rk_bst_small_forward call (every array it points into is part of
    the tuple, so holding the tuple keeps them alive; the tensors stay the caller's)."""
    B, T = seq.shape
    params = (ctypes.c_void_p * (BST_BLOCK_PARAMS * len(blocks)))()
    scalars = (ctypes.c_float * (3 * len(blocks)))()
    for i, (tensors, sc) in enumerate(blocks):
        for k, t in enumerate(tensors):
            params[BST_BLOCK_PARAMS * i + k] = ptr(t)
        for k in range(3):
            scalars[3 * i + k] = float(sc[k])
    arr = _seg_array(segs)
    larr = (_lib.MlpLayer * max(1, len(layers)))(*layers)
    return (arr, len(segs), width, ptr(table), table.shape[0], table.stride(0), ptr(seq), seq.stride(0), T,
            ptr(seq_len), B, heads, len(blocks), params, scalars, 1 if pool_mean else 0, larr, len(layers),
            ctypes.byref(head), _lib.stream_of(table))


def bst_small_forward(segs, width, table, seq, seq_len, heads, blocks, pool_mean, layers, head: Epilogue) -> bool:
    """rk_bst_small_forward: the whole BST eval forward at d_model 16 in one launch.  False (nothing
    launched) outside its envelope (RK_ERR_UNSUPPORTED), for the three-launch path."""
    rc = _lib.load().rk_bst_small_forward(*bst_small_forward_args(segs, width, table, seq, seq_len, heads, blocks,
                                                                  pool_mean, layers, head))
    if rc == _lib.RK_ERR_UNSUPPORTED:
        return False
    check(rc, "rk_bst_small_forward")
    return True


def bn_fold(mean, var, weight, bias, eps, scale, shift):
    lib = _lib.load()
    check(lib.rk_bn_fold(ptr(mean), ptr(var), ptr(weight), ptr(bias), float(eps), mean.numel(), ptr(scale),
                         ptr(shift), _lib.stream_of(mean)), "rk_bn_fold")


_EPI_PTR_FIELDS = {f for f, t in Epilogue._fields_ if t is ctypes.c_void_p}


def make_epilogue(**kw) -> Epilogue:
    ep = Epilogue()
    for k, v in kw.items():
        if v is None:
            continue
        if k == "act" and isinstance(v, str):
            v = ACT[v]
        if k in _EPI_PTR_FIELDS and isinstance(v, torch.Tensor):
            v = v.data_ptr()
        setattr(ep, k, v)
    return ep


_MLP_PTR_FIELDS = {f for f, t in _lib.MlpLayer._fields_ if t is ctypes.c_void_p}


def pack_mlp_weight(weight: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """[n, k] nn.Linear weight -> the zero-padded [pad64(n), pad64(k)] layout rk_mlp_forward reads
    (into `out` when given: a previous image of the same weight shape, rewritten in place)."""
    lib = _lib.load()
    n, k = weight.shape
    rows, cols = (n + 63) // 64 * 64, (k + 63) // 64 * 64  # rk_mlp_packed_size
    if out is None or tuple(out.shape) != (rows, cols) or out.device != weight.device:
        out = torch.empty(rows, cols, device=weight.device, dtype=torch.float32)
    w = weight.detach()
    if w.stride(1) != 1:
        w = w.contiguous()
    check(lib.rk_mlp_pack_weight(w.data_ptr(), w.stride(0), n, k, out.data_ptr(), _lib.stream_of(out)),
          "rk_mlp_pack_weight")
    return out


def make_mlp_layer(weight: torch.Tensor, packed: torch.Tensor, **kw) -> "_lib.MlpLayer":
    """One fused-MLP layer: `weight` the [n, k] parameter (n is taken from it), `packed` its
    pack_mlp_weight() image."""
    L = _lib.MlpLayer()
    L.w, L.ldw, L.n = packed.data_ptr(), packed.stride(0), weight.shape[0]
    for k, v in kw.items():
        if v is None:
            continue
        if k == "act" and isinstance(v, str):
            v = ACT[v]
        if k in _MLP_PTR_FIELDS and isinstance(v, torch.Tensor):
            v = v.data_ptr()
        setattr(L, k, v)
    return L


def mlp_forward(x: torch.Tensor, layers, head: Epilogue = None, out: torch.Tensor = None, *, K0: int = None):
    """Whole MLP tail (all hidden layers + optional Linear(N,1)+sigmoid head) in one launch."""
    lib = _lib.load()
    arr = (_lib.MlpLayer * max(1, len(layers)))(*layers)
    K0 = x.shape[1] if K0 is None else K0
    check(lib.rk_mlp_forward(x.data_ptr(), x.stride(0), x.shape[0], K0, arr, len(layers),
                             ctypes.byref(head) if head is not None else None, ptr(out),
                             out.stride(0) if out is not None else 0, _lib.stream_of(x)), "rk_mlp_forward")
    return out


def linear_tiled(x: torch.Tensor, layer: "_lib.MlpLayer", out: torch.Tensor, K: int = None):
    """One packed MLP layer as a 2D-tiled GEMM (rk_linear_tiled) into `out` [M, n]."""
    lib = _lib.load()
    K = x.shape[1] if K is None else K
    check(lib.rk_linear_tiled(x.data_ptr(), x.stride(0), x.shape[0], K, ctypes.byref(layer), out.data_ptr(),
                              out.stride(0), _lib.stream_of(x)), "rk_linear_tiled")
    return out


_DIN_L2_WS = {}


def _din_l2_workspace(device, batch):
    """rk_din_forward's l2 workspace: ceil(batch/16) partials + a completion counter that starts at
    zero and that every launch leaves at zero, so it is allocated (zeroed) once per device and
    size and reused, also by a hipGraph captured after a warm-up call.  Eager DIN forwards of one
    batch size on one device therefore must not run concurrently on two streams (prepared plans
    carry their own: din_forward_plan)."""
    n = (batch + 15) // 16 + 1
    key = (str(torch.device(device)), n)
    ws = _DIN_L2_WS.get(key)
    if ws is None:
        ws = torch.zeros(n, device=device, dtype=torch.float32)
        _DIN_L2_WS[key] = ws
    return ws


def din_pack_attention(att_weights, H: int) -> torch.Tensor:
    """rk_din_pack_attention: the split attention weights as din_forward_kernel's LDS image."""
    lib = _lib.load()
    w1, b1, w2, b2, w3, _ = att_weights
    _lib.ensure_device(w1.device)
    n = lib.rk_din_attention_image_floats(H)
    if n <= 0:
        raise ValueError(f"rankops.din_pack_attention: H={H} not in (8, 16, 32)")
    img = torch.empty(n, device=w1.device, dtype=torch.float32)
    check(lib.rk_din_pack_attention(ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(w3), H, ptr(img),
                                    _lib.stream_of(img)), "rk_din_pack_attention")
    return img


def _din_forward_args(segs, width, q_col, att_col, key_table, seq, seq_len, H, att_weights, use_softmax, layers,
                      head: Epilogue, batch, device, l2_col0, l2_scale, l2_out, att_image, private_ws=False):
    """The rk_din_forward argument list (without the stream) and the ctypes arrays it points into.
    private_ws: an l2 workspace of its own (a prepared plan, which may run concurrently with other
    plans on other streams) instead of the shared per-(device, batch) one."""
    w1, b1, w2, b2, w3, b3 = att_weights
    arr = _seg_array(segs)
    larr = (_lib.MlpLayer * max(1, len(layers)))(*layers)
    ws = None
    if l2_out is not None:
        if private_ws:
            ws = torch.zeros((batch + 15) // 16 + 1, device=device, dtype=torch.float32)
            torch.cuda.current_stream(ws.device).synchronize()  # zeroed before a launch on any stream
        else:
            ws = _din_l2_workspace(device, batch)
    args = (arr, len(segs), width, q_col, att_col, ptr(key_table), key_table.shape[0], key_table.stride(0), ptr(seq),
            seq.stride(0), seq.shape[1], ptr(seq_len), batch, H, ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(w3),
            ptr(b3), 1 if use_softmax else 0, larr, len(layers), ctypes.byref(head), l2_col0, float(l2_scale),
            ptr(ws), ptr(l2_out), ptr(att_image))
    return args, (arr, larr, head, ws)


def din_forward(segs, width, q_col, att_col, key_table, seq, seq_len, H, att_weights, use_softmax, layers,
                head: Epilogue, batch, device, l2_col0=0, l2_scale=0.0, l2_out=None, att_image=None):
    """Whole DIN eval forward (row gather, attention, fcn tail, head, l2 partials) in one launch."""
    lib = _lib.load()
    _lib.ensure_device(device)
    args, _keep = _din_forward_args(segs, width, q_col, att_col, key_table, seq, seq_len, H, att_weights,
                                    use_softmax, layers, head, batch, device, l2_col0, l2_scale, l2_out, att_image)
    check(lib.rk_din_forward(*args, _lib.raw_stream(device)), "rk_din_forward")


def pack_epilogue_image(larr, nlayers, K0, device):
    """The per-column epilogue parameters of a layer stack with a compiled streamed plan, packed
    in the streamed tail's LDS layout (rk_mlp_pack_epilogue), or None (no plan;
    RANKOPS_DIN_EPI_DMA=0: the DIN kernel resolves them per column at launch instead)."""
    lib = _lib.load()
    n = lib.rk_mlp_epilogue_image_floats(larr, nlayers, K0)
    if n <= 0 or os.environ.get("RANKOPS_DIN_EPI_DMA", "1") == "0":
        return None
    img = torch.empty(n, device=device, dtype=torch.float32)
    check(lib.rk_mlp_pack_epilogue(larr, nlayers, K0, img.data_ptr(), _lib.raw_stream(device)), "rk_mlp_pack_epilogue")
    return img


class DinPlan:
    """rk_din_forward_plan: the fused DIN forward with its arguments validated once; calling it
    launches the kernel on the current stream (one launch, no per-call host work besides the
    ctypes call).  Binds the pointers it was made with — `keep` holds every tensor it reads or
    writes alive for the plan's lifetime."""

    def __init__(self, args, keep, device):
        self._lib = _lib.load()
        self._device = device
        self._handle = ctypes.c_void_p()
        check(self._lib.rk_din_forward_plan(*args, ctypes.byref(self._handle)), "rk_din_forward_plan")
        self._keep = keep
        self._epi = None
        # phase B's epilogue parameters packed once (rk_mlp_pack_epilogue) and copied into LDS by
        # the kernel, for plans whose launches use them (balanced streamed plans); the image is a
        # snapshot of the current BatchNorm / Dice parameters, as the plan binds the weights
        larr, nl, width = args[21], args[22], args[2]
        img = pack_epilogue_image(larr, nl, width, device)
        if img is not None and self._lib.rk_din_plan_set_epilogue_image(self._handle, img.data_ptr()) == _lib.RK_OK:
            self._epi = img  # (RK_ERR_UNSUPPORTED: no streamed phase B)

    def launch(self):
        check(self._lib.rk_din_plan_launch(self._handle, _lib.raw_stream(self._device)),
              "rk_din_plan_launch")

    def launch_on(self, stream: int):
        """Launch on an explicit HIP stream (a raw handle, e.g. `torch.cuda.Stream().cuda_stream`),
        without making it the current stream."""
        check(self._lib.rk_din_plan_launch(self._handle, ctypes.c_void_p(stream)), "rk_din_plan_launch")

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            self._lib.rk_din_plan_destroy(h)
            h.value = None


def din_forward_plan(segs, width, q_col, att_col, key_table, seq, seq_len, H, att_weights, use_softmax, layers,
                     head: Epilogue, batch, device, l2_col0=0, l2_scale=0.0, l2_out=None, att_image=None, keep=()):
    _lib.ensure_device(device)
    args, k = _din_forward_args(segs, width, q_col, att_col, key_table, seq, seq_len, H, att_weights, use_softmax,
                                layers, head, batch, device, l2_col0, l2_scale, l2_out, att_image, private_ws=True)
    return DinPlan(args, (k, tuple(keep)), device)


def linear(x: torch.Tensor, weight: torch.Tensor, out: torch.Tensor = None, *, M: int = None, K: int = None,
           x_ptr: int = None, ldx: int = None, x_periodic: torch.Tensor = None, x_period: int = 0,
           y_ptr: int = None, ldy: int = None, epilogue: Epilogue = None):
    """y = epilogue(x . weight^T) on FP32 MFMA.  weight is [N, K] (nn.Linear layout)."""
    lib = _lib.load()
    N = weight.shape[0]
    K = weight.shape[1] if K is None else K
    M = x.shape[0] if M is None else M
    if weight.stride(1) != 1:
        raise ValueError("rankops.linear: weight needs unit column stride")
    xp = x.data_ptr() if x_ptr is None else x_ptr
    lx = x.stride(0) if ldx is None else ldx
    if y_ptr is None and out is not None:
        y_ptr, ldy = out.data_ptr(), out.stride(0) if ldy is None else ldy
    ep = epilogue if epilogue is not None else Epilogue()
    check(lib.rk_linear(xp, lx, ptr(x_periodic), x_period, weight.data_ptr(), weight.stride(0), M, N, K,
                        ctypes.byref(ep), y_ptr, ldy or 0, _lib.stream_of(x)), "rk_linear")
    return out


# ---------------------------------------------------------------- training (§8(f) #2)

_WS_FLOATS = {}
_WS = {}


def _wgrad_ws_floats(lib, M, N, R):
    key = (M, N, R)
    n = _WS_FLOATS.get(key)
    if n is None:
        n = _WS_FLOATS[key] = lib.rk_gemm_wgrad_workspace_floats(M, N, R)
    return n


def _wgrad_workspace(nws: int, device, stream: int) -> torch.Tensor:
    """rk_gemm_wgrad scratch: one buffer per (device, stream) reused by every eager call (calls on
    one stream are ordered, and a launch reads only what it wrote); under stream capture a fresh
    allocation from the graph's pool, so a replay never shares scratch with eager work."""
    if torch.cuda.is_current_stream_capturing():
        return torch.empty(nws, device=device, dtype=torch.float32)
    key = (device, stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < nws:
        ws = _WS[key] = torch.empty(max(nws, 1 << 16), device=device, dtype=torch.float32)
    return ws


def gemm(trans_a: bool, trans_b: bool, M: int, N: int, R: int, A: torch.Tensor, lda: int, B: torch.Tensor, ldb: int,
         C: torch.Tensor, ldc: int = None, *, A_mask: torch.Tensor = None, row_sums: torch.Tensor = None,
         accumulate: bool = False, split: int = 0):
    """C[m, n] (+)= sum_r opA(m, r) opB(n, r) (rk_gemm; layouts in include/rankops.h).  Weight
    gradients (both operands transposed: dW = dZ^T X over the batch rows) go to rk_gemm_wgrad when
    the layout allows it."""
    lib = _lib.load()
    ldc_ = C.stride(0) if ldc is None else ldc
    if (trans_a and trans_b and split <= 0 and R >= 512 and (M | N | lda | ldb | ldc_) % 4 == 0
            and all(t is None or t.data_ptr() % 16 == 0 for t in (A, B, A_mask, C, row_sums))):
        nws = _wgrad_ws_floats(lib, M, N, R)
        st = _lib.stream_of(C)
        ws = _wgrad_workspace(nws, C.device, st)
        check(lib.rk_gemm_wgrad(M, N, R, ptr(A), lda, ptr(A_mask), ptr(B), ldb, ptr(C), ldc_, ptr(row_sums),
                                int(accumulate), ptr(ws), nws, st), "rk_gemm_wgrad")
        return C
    check(lib.rk_gemm(int(trans_a), int(trans_b), M, N, R, ptr(A), lda, ptr(A_mask), ptr(B), ldb, ptr(C),
                      C.stride(0) if ldc is None else ldc, ptr(row_sums), int(accumulate), split,
                      _lib.stream_of(C)), "rk_gemm")
    return C


def linear_backward(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, *, relu_out: torch.Tensor = None,
                    need_dx: bool = True, dx: torch.Tensor = None):
    """nn.Linear (+ ReLU when relu_out = the layer's post-ReLU output) backward:
    dz = dy * [relu_out > 0]; dW = dz^T x; db = sum_b dz; dx = dz W.  -> (dx, dW, db)."""
    Bsz, N = dy.shape
    K = weight.shape[1]
    if relu_out is not None and (relu_out.shape != dy.shape or relu_out.stride() != dy.stride()):
        raise ValueError("rankops.linear_backward: relu_out must have dy's shape and strides")
    dW = torch.empty(N, K, device=dy.device, dtype=torch.float32)
    db = torch.empty(N, device=dy.device, dtype=torch.float32)
    gemm(True, True, N, K, Bsz, dy, dy.stride(0), x, x.stride(0), dW, A_mask=relu_out, row_sums=db)
    if need_dx:
        if dx is None:
            dx = torch.empty(Bsz, K, device=dy.device, dtype=torch.float32)
        gemm(False, True, Bsz, K, N, dy, dy.stride(0), weight, weight.stride(0), dx, A_mask=relu_out)
    return dx, dW, db


def logit_head_backward(dlogit, dprob, prob, xa, xb, w, dxa, dxb, dw, db, g_out=None):
    lib = _lib.load()
    check(lib.rk_logit_head_backward(ptr(dlogit), ptr(dprob), ptr(prob), xa.shape[0], ptr(xa), xa.stride(0),
                                     xa.shape[1], ptr(xb), xb.stride(0) if xb is not None else 0,
                                     xb.shape[1] if xb is not None else 0, ptr(w), ptr(dxa),
                                     dxa.stride(0) if dxa is not None else 0, ptr(dxb),
                                     dxb.stride(0) if dxb is not None else 0, ptr(dw), ptr(db), ptr(g_out),
                                     _lib.stream_of(xa)), "rk_logit_head_backward")


def relu_backward(dy, y, out, accumulate=False):
    lib = _lib.load()
    if not (dy.is_contiguous() and y.is_contiguous() and out.is_contiguous()) or dy.shape != y.shape != out.shape:
        raise ValueError("rankops.relu_backward: contiguous tensors of one shape expected")
    check(lib.rk_relu_backward(ptr(dy), ptr(y), ptr(out), dy.numel(), int(accumulate), _lib.stream_of(dy)),
          "rk_relu_backward")
    return out


def dcn_cross_backward(x0, cross_w, cross_b, num_layers, dxl, dx0, accumulate=True):
    lib = _lib.load()
    check(lib.rk_dcn_cross_backward(ptr(x0), x0.stride(0), x0.shape[0], x0.shape[1], ptr(cross_w), ptr(cross_b),
                                    num_layers, ptr(dxl), dxl.stride(0), ptr(dx0), dx0.stride(0), int(accumulate),
                                    _lib.stream_of(x0)), "rk_dcn_cross_backward")


def embedding_backward(grad_segs, batch, dx):
    lib = _lib.load()
    check(lib.rk_embedding_backward(_as_seg_array(grad_segs), len(grad_segs), batch, ptr(dx), dx.stride(0),
                                    _lib.stream_of(dx)), "rk_embedding_backward")


def embedding_backward_seq(grad, seq, dx):
    """rk_embedding_backward_seq: grad[seq[b, t]] += dx[b*T + t] with runs of equal consecutive ids
    pre-summed (no sort); False (nothing launched) when the layout does not allow it."""
    B, T = seq.shape
    d = grad.shape[1]
    if (d % 2 or d > 128 or dx.stride(0) % 2 or grad.stride(0) % 2 or seq.stride(1) != 1
            or dx.data_ptr() % 8 or grad.data_ptr() % 8):
        return False
    lib = _lib.load()
    seg = table_segment(grad, seq, 0, idx_stride=seq.stride(0))
    check(lib.rk_embedding_backward_seq(ctypes.byref(seg), B, T, ptr(dx), dx.stride(0), _lib.stream_of(dx)),
          "rk_embedding_backward_seq")
    return True


def embedding_backward_sorted(grad_seg, n, dx):
    """rk_embedding_backward_sorted: one table segment over n index entries (sorted segment-reduce)."""
    lib = _lib.load()
    nbytes = ctypes.c_int64()
    check(lib.rk_embedding_backward_sorted_workspace_size(n, ctypes.byref(nbytes)),
          "rk_embedding_backward_sorted_workspace_size")
    ws = torch.empty(max(1, nbytes.value), device=dx.device, dtype=torch.uint8)
    check(lib.rk_embedding_backward_sorted(ctypes.byref(grad_seg), n, ptr(dx), dx.stride(0), ptr(ws), nbytes.value,
                                           _lib.stream_of(dx)), "rk_embedding_backward_sorted")


def adam_step(entries, lr, beta1, beta2, eps, weight_decay, step, stream):
    """entries: list of (param, grad, exp_avg, exp_avg_sq[, device step tensor]) float32 tensors."""
    lib = _lib.load()
    arr = (_lib.AdamTensor * len(entries))(*[
        _lib.AdamTensor(e[0].data_ptr(), e[1].data_ptr(), e[2].data_ptr(), e[3].data_ptr(), e[0].numel(),
                        e[4].data_ptr() if len(e) > 4 else None) for e in entries])
    check(lib.rk_adam_step(arr, len(entries), lr, beta1, beta2, eps, weight_decay, step, stream), "rk_adam_step")


def rng_next(counter: torch.Tensor, slot: torch.Tensor):
    lib = _lib.load()
    check(lib.rk_rng_next(ptr(counter), ptr(slot), _lib.stream_of(counter)), "rk_rng_next")


def dropout_mask(seed: int, slot: torch.Tensor, batch: int, n: int, p: float) -> torch.Tensor:
    lib = _lib.load()
    out = torch.empty(batch, n, device=slot.device, dtype=torch.float32)
    check(lib.rk_dropout_mask(seed, ptr(slot), batch, n, p, ptr(out), _lib.stream_of(out)), "rk_dropout_mask")
    return out


def _act_code(act):
    """True/False (ReLU or none) or an ACT name."""
    if isinstance(act, str):
        return ACT[act]
    return _lib.RK_ACT_RELU if act else _lib.RK_ACT_NONE


def _stats_updated(bn):
    """After a train-mode kernel updated `bn`'s running statistics through raw pointers: count the
    batch as torch's BatchNorm does and bump the buffers' versions so eval-mode folds
    (common.FoldedBN) keyed on them recompute."""
    if bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    torch.autograd.graph.increment_version([bn.running_mean, bn.running_var])


def bn_act_train_forward(z, bias, bn, act, p, seed, slot, y, save_mean, save_invstd, workspace, slope=0.0):
    """bn: an nn.BatchNorm1d (train mode) or None; act: True (ReLU), False, or 'leaky' with `slope`."""
    lib = _lib.load()
    track = bn is not None and bn.track_running_stats and bn.running_mean is not None
    check(lib.rk_bn_act_train_forward(
        ptr(z), z.stride(0), z.shape[0], z.shape[1], ptr(bias), int(bn is not None),
        ptr(bn.weight) if bn is not None else None, ptr(bn.bias) if bn is not None else None,
        float(bn.eps) if bn is not None else 0.0, float(bn.momentum) if bn is not None else 0.0,
        ptr(bn.running_mean) if track else None, ptr(bn.running_var) if track else None, ptr(workspace),
        ptr(save_mean), ptr(save_invstd), _act_code(act), float(slope), float(p), seed, ptr(slot), ptr(y),
        y.stride(0), _lib.stream_of(z)), "rk_bn_act_train_forward")
    if track:
        _stats_updated(bn)


def bn_act_backward(dy, z, bias, bn, act, p, seed, slot, save_mean, save_invstd, workspace, dz, dgamma, dbeta,
                    slope=0.0):
    lib = _lib.load()
    check(lib.rk_bn_act_backward(
        ptr(dy), dy.stride(0), ptr(z), z.stride(0), z.shape[0], z.shape[1], ptr(bias), int(bn is not None),
        ptr(bn.weight) if bn is not None else None, ptr(bn.bias) if bn is not None else None, ptr(save_mean),
        ptr(save_invstd), _act_code(act), float(slope), float(p), seed, ptr(slot), ptr(workspace), ptr(dz), dz.stride(0), ptr(dgamma),
        ptr(dbeta), _lib.stream_of(dy)), "rk_bn_act_backward")


def dice_train_forward(z, bias, dice, y, save_mean, save_invstd, workspace):
    """Dice (din.py:26-36) with batch statistics on z + bias; `dice` is the Dice module (its .bn
    running statistics and num_batches_tracked are updated as torch's train-mode BatchNorm does)."""
    lib = _lib.load()
    bn = dice.bn
    track = bn.track_running_stats and bn.running_mean is not None
    check(lib.rk_dice_train_forward(ptr(z), z.stride(0), z.shape[0], z.shape[1], ptr(bias), ptr(dice.alpha),
                                    float(bn.eps), float(bn.momentum), ptr(bn.running_mean) if track else None,
                                    ptr(bn.running_var) if track else None, ptr(workspace), ptr(save_mean),
                                    ptr(save_invstd), ptr(y), y.stride(0), _lib.stream_of(z)), "rk_dice_train_forward")
    if track:
        _stats_updated(bn)


def dice_backward(dy, z, bias, dice, save_mean, save_invstd, workspace, dz, dalpha):
    lib = _lib.load()
    check(lib.rk_dice_backward(ptr(dy), dy.stride(0), ptr(z), z.stride(0), z.shape[0], z.shape[1], ptr(bias),
                               ptr(dice.alpha), ptr(save_mean), ptr(save_invstd), ptr(workspace), ptr(dz),
                               dz.stride(0), ptr(dalpha), _lib.stream_of(dy)), "rk_dice_backward")


def prelu_train_forward(z, bias, prelu, y):
    """nn.PReLU (din.py:277-279) on z + bias; `prelu` is the module (its weight stays on the device)."""
    lib = _lib.load()
    w = prelu.weight
    check(lib.rk_prelu_train_forward(ptr(z), z.stride(0), z.shape[0], z.shape[1], ptr(bias), ptr(w), w.numel(),
                                     ptr(y), y.stride(0), _lib.stream_of(z)), "rk_prelu_train_forward")


def prelu_backward(dy, z, bias, prelu, workspace, dz, dweight):
    lib = _lib.load()
    w = prelu.weight
    check(lib.rk_prelu_backward(ptr(dy), dy.stride(0), ptr(z), z.stride(0), z.shape[0], z.shape[1], ptr(bias), ptr(w),
                                w.numel(), ptr(workspace), ptr(dz), dz.stride(0), ptr(dweight), _lib.stream_of(dy)),
          "rk_prelu_backward")


def din_att_cross(x, q_col, key_table, seq, T, H, keys, cross):
    lib = _lib.load()
    check(lib.rk_din_att_cross(ptr(x), x.stride(0), q_col, ptr(key_table), key_table.shape[0], key_table.stride(0),
                               ptr(seq), seq.stride(0), x.shape[0], T, H, ptr(keys), ptr(cross),
                               _lib.stream_of(x)), "rk_din_att_cross")


def din_att_pool_forward(a2, w3, b3, keys, seq_len, T, H, softmax, weights, x, att_col):
    lib = _lib.load()
    check(lib.rk_din_att_pool_forward(ptr(a2), a2.shape[1], ptr(w3), ptr(b3), ptr(keys), ptr(seq_len), x.shape[0],
                                      T, H, int(bool(softmax)), ptr(weights), ptr(x), x.stride(0), att_col,
                                      _lib.stream_of(x)), "rk_din_att_pool_forward")


def din_att_pool_backward(dx, att_col, weights, keys, a2, w3, seq_len, T, H, softmax, dkeys, da2):
    lib = _lib.load()
    check(lib.rk_din_att_pool_backward(ptr(dx), dx.stride(0), att_col, ptr(weights), ptr(keys), ptr(a2),
                                       a2.shape[1], ptr(w3), ptr(seq_len), dx.shape[0], T, H, int(bool(softmax)),
                                       ptr(dkeys), ptr(da2), _lib.stream_of(dx)), "rk_din_att_pool_backward")


def din_cross_fold(dcross, x, q_col, keys, T, H, dkeys, dx):
    lib = _lib.load()
    check(lib.rk_din_cross_fold(ptr(dcross), ptr(x), x.stride(0), q_col, ptr(keys), x.shape[0], T, H, ptr(dkeys),
                                ptr(dx), dx.stride(0), _lib.stream_of(dx)), "rk_din_cross_fold")


def row_l2norm_backward(x, col0, ncols, scale, grad_out, dx):
    lib = _lib.load()
    check(lib.rk_row_l2norm_backward(ptr(x), x.stride(0), x.shape[0], col0, ncols, float(scale), ptr(grad_out),
                                     ptr(dx), dx.stride(0), _lib.stream_of(dx)), "rk_row_l2norm_backward")


def fwfm_backward(emb_segs, dim, batch, field_weight, prob, dprob, d_emb, dz, d_field_weight, d_bias):
    lib = _lib.load()
    check(lib.rk_fwfm_backward(_as_seg_array(emb_segs), len(emb_segs), dim, batch, ptr(field_weight), ptr(prob),
                               ptr(dprob), ptr(d_emb), d_emb.stride(0), ptr(dz), ptr(d_field_weight), ptr(d_bias),
                               _lib.stream_of(prob)), "rk_fwfm_backward")


def afm_pairs(fields, dim, batch, emb, pairs):
    lib = _lib.load()
    check(lib.rk_afm_pairs(_seg_array(fields), len(fields), dim, batch, ptr(emb), ptr(pairs), _lib.stream_of(emb)),
          "rk_afm_pairs")


def afm_pool_forward(a1, w2, b2, pairs, num_pairs, dim, dense, wd, bd, wp, bp, weights, ws, logit, pred):
    lib = _lib.load()
    check(lib.rk_afm_pool_forward(ptr(a1), a1.shape[1], ptr(w2), ptr(b2), ptr(pairs), num_pairs, dim, ptr(dense),
                                  dense.stride(0), dense.shape[1], ptr(wd), ptr(bd), ptr(wp), ptr(bp), dense.shape[0],
                                  ptr(weights), ptr(ws), ptr(logit), ptr(pred), _lib.stream_of(pred)),
          "rk_afm_pool_forward")


def afm_pool_backward(dpred, dtotal, pred, weights, ws, pairs, a1, w2, wp, dense, num_pairs, dim, d_pairs, da1, acc):
    lib = _lib.load()
    check(lib.rk_afm_pool_backward(ptr(dpred), ptr(dtotal), ptr(pred), ptr(weights), ptr(ws), ptr(pairs), ptr(a1),
                                   a1.shape[1], ptr(w2), ptr(wp), ptr(dense), dense.stride(0), dense.shape[1],
                                   dense.shape[0], num_pairs, dim, ptr(d_pairs), ptr(da1), ptr(acc),
                                   _lib.stream_of(pred)), "rk_afm_pool_backward")


def afm_pair_fold(d_pairs, emb, num_fields, dim, d_emb):
    lib = _lib.load()
    check(lib.rk_afm_pair_fold(ptr(d_pairs), ptr(emb), num_fields, dim, emb.shape[0], ptr(d_emb),
                               _lib.stream_of(emb)), "rk_afm_pair_fold")


def bst_add_pos(x, pos, T, xp):
    lib = _lib.load()
    check(lib.rk_bst_add_pos(ptr(x), ptr(pos), T, x.shape[0], x.shape[1], ptr(xp), _lib.stream_of(x)),
          "rk_bst_add_pos")


def bst_gather_pos(table, idx, T, pos, x, xp):
    """x = table[idx], xp = x + pos[m % T] in one pass (rk_bst_gather_pos); False when the layout
    does not allow it (nothing launched)."""
    d = table.shape[1]
    if (d % 4 or table.stride(0) % 4 or idx.stride(0) != 1 or pos.stride(0) != d
            or any(t.data_ptr() % 16 for t in (table, pos, x, xp))):
        return False
    lib = _lib.load()
    check(lib.rk_bst_gather_pos(ptr(table), table.shape[0], table.stride(0), ptr(idx), idx.shape[0], T, d, ptr(pos),
                                ptr(x), ptr(xp), _lib.stream_of(x)), "rk_bst_gather_pos")
    return True


def bst_attn_train_forward(qkv, B, T, d, heads, seq_len, probs, ctx):
    lib = _lib.load()
    check(lib.rk_bst_attn_train_forward(ptr(qkv), B, T, d, heads, ptr(seq_len), ptr(probs), ptr(ctx),
                                        _lib.stream_of(qkv)), "rk_bst_attn_train_forward")


def bst_attn_train_backward(qkv, probs, dctx, B, T, d, heads, dqkv):
    lib = _lib.load()
    check(lib.rk_bst_attn_train_backward(ptr(qkv), ptr(probs), ptr(dctx), B, T, d, heads, ptr(dqkv),
                                         _lib.stream_of(qkv)), "rk_bst_attn_train_backward")


def linear_res_dropout_ln(x, weight, bias, base, p, seed, slot, ln, r, y, mean, rstd) -> bool:
    """rk_linear_res_dropout_ln: y = LayerNorm(base + dropout(x W^T + bias)) in one launch; False
    (nothing launched) when the shape is not the fused kernel's (d_model != 128, K, alignment, M)."""
    d = weight.shape[0]
    if (d != 128 or weight.shape[1] != x.shape[1] or weight.stride(1) != 1 or x.stride(1) != 1
            or not all(t.is_contiguous() for t in (base, r, y)) or ln.weight is None or ln.bias is None):
        return False
    lib = _lib.load()
    rc = lib.rk_linear_res_dropout_ln(ptr(x), x.stride(0), x.shape[0], x.shape[1], ptr(weight), weight.stride(0),
                                      ptr(bias), ptr(base), float(p), seed, ptr(slot), ptr(ln.weight), ptr(ln.bias),
                                      float(ln.eps), ptr(r), ptr(y), ptr(mean), ptr(rstd), _lib.stream_of(x))
    if rc == _lib.RK_ERR_UNSUPPORTED:
        return False
    check(rc, "rk_linear_res_dropout_ln")
    return True


def bst_res_dropout_ln_forward(base, o, p, seed, slot, ln, r, y, mean, rstd):
    lib = _lib.load()
    check(lib.rk_bst_res_dropout_ln_forward(ptr(base), ptr(o), base.shape[0], base.shape[1], float(p), seed,
                                            ptr(slot), ptr(ln.weight), ptr(ln.bias), float(ln.eps), ptr(r), ptr(y),
                                            ptr(mean), ptr(rstd), _lib.stream_of(base)),
          "rk_bst_res_dropout_ln_forward")


def bst_ln_backward(dy, r, mean, rstd, ln, p, seed, slot, dr, d_o, dgamma, dbeta):
    lib = _lib.load()
    nws = lib.rk_bst_ln_backward_workspace_floats(r.shape[1])
    ws = torch.empty(nws, device=r.device, dtype=torch.float32)
    check(lib.rk_bst_ln_backward(ptr(dy), ptr(r), ptr(mean), ptr(rstd), ptr(ln.weight), r.shape[0], r.shape[1],
                                 float(p), seed, ptr(slot), ptr(dr), ptr(d_o), ptr(dgamma), ptr(dbeta), ptr(ws),
                                 nws, _lib.stream_of(dy)), "rk_bst_ln_backward")


def bst_pool_ln_backward(drow, col, T, seq_len, mean_pool, r, mean, rstd, ln, p, seed, slot, dr, d_o, dgamma,
                         dbeta):
    """bst_ln_backward whose incoming gradient is the pooling backward's broadcast of drow
    (rk_bst_pool_ln_backward); returns False (nothing launched) when the layout does not allow it."""
    lib = _lib.load()
    d = r.shape[1]
    if d % 4 or any(t is not None and t.data_ptr() % 16 for t in (r, ln.weight, dr, d_o)):
        return False
    nws = lib.rk_bst_ln_backward_workspace_floats(d)
    ws = torch.empty(nws, device=r.device, dtype=torch.float32)
    check(lib.rk_bst_pool_ln_backward(ptr(drow), drow.stride(0), col, T, ptr(seq_len), int(mean_pool), ptr(r),
                                      ptr(mean), ptr(rstd), ptr(ln.weight), r.shape[0], d, float(p), seed, ptr(slot),
                                      ptr(dr), ptr(d_o), ptr(dgamma), ptr(dbeta), ptr(ws), nws, _lib.stream_of(r)),
          "rk_bst_pool_ln_backward")
    return True


def bst_pos_backward(dxp, B, T, dpos):
    lib = _lib.load()
    check(lib.rk_bst_pos_backward(ptr(dxp), B, T, dxp.shape[1], ptr(dpos), _lib.stream_of(dxp)),
          "rk_bst_pos_backward")


def bst_leaky_dropout(inp, f, slope, p, seed, slot, backward, out):
    lib = _lib.load()
    check(lib.rk_bst_leaky_dropout(ptr(inp), ptr(f), f.numel(), float(slope), float(p), seed, ptr(slot),
                                   int(backward), ptr(out), _lib.stream_of(f)), "rk_bst_leaky_dropout")


def bst_pool(x, B, T, seq_len, mean, row, col):
    lib = _lib.load()
    check(lib.rk_bst_pool(ptr(x), B, T, x.shape[1], ptr(seq_len), int(mean), ptr(row), row.stride(0), col,
                          _lib.stream_of(x)), "rk_bst_pool")


def bst_pool_backward(drow, col, B, T, d, seq_len, mean, dx):
    lib = _lib.load()
    check(lib.rk_bst_pool_backward(ptr(drow), drow.stride(0), col, B, T, d, ptr(seq_len), int(mean), ptr(dx),
                                   _lib.stream_of(dx)), "rk_bst_pool_backward")


def fm_backward(deep_in, d_deep, dfm2, num_fields, dim, out):
    lib = _lib.load()
    check(lib.rk_fm_backward(ptr(deep_in), deep_in.stride(0), ptr(d_deep), d_deep.stride(0) if d_deep is not None else 0,
                             ptr(dfm2), deep_in.shape[0], num_fields, dim, ptr(out), out.stride(0),
                             _lib.stream_of(deep_in)), "rk_fm_backward")


def fm_combine_backward(dprob, dtotal, dfm1_in, dfm2_in, ddeep_in, prob, fm1, fm2, deep, final_w, dfm1, dfm2, ddeep,
                        dfinal_w, dfinal_b):
    lib = _lib.load()
    check(lib.rk_fm_combine_backward(ptr(dprob), ptr(dtotal), ptr(dfm1_in), ptr(dfm2_in), ptr(ddeep_in), ptr(prob),
                                     ptr(fm1), ptr(fm2), ptr(deep), ptr(final_w), prob.shape[0], ptr(dfm1), ptr(dfm2),
                                     ptr(ddeep), ptr(dfinal_w), ptr(dfinal_b), _lib.stream_of(prob)),
          "rk_fm_combine_backward")
