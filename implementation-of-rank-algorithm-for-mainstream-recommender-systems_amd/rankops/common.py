"""Plumbing shared by the drop-in models: vocab sizes, per-call random weights (H2),
BatchNorm folding, packed-weight caches and the fused MLP tail."""
from __future__ import annotations

import math
import os
import weakref
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn

from . import ops

WECHAT_VOCAB_FILES = {
    "userid": "userid.txt",
    "feedid": "feedid.txt",
    "device": "device.txt",
    "authorid": "authorid.txt",
    "bgm_song_id": "bgm_song_id.txt",
    "bgm_singer_id": "bgm_singer_id.txt",
    "manual_tag_list": "manual_tag_id.txt",
}

DENSE_FEATURES = [
    "videoplayseconds", "u_read_comment_7d_sum", "u_like_7d_sum",
    "u_click_avatar_7d_sum", "u_forward_7d_sum", "u_comment_7d_sum",
    "u_follow_7d_sum", "u_favorite_7d_sum", "i_read_comment_7d_sum",
    "i_like_7d_sum", "i_click_avatar_7d_sum", "i_forward_7d_sum",
    "i_comment_7d_sum", "i_follow_7d_sum", "i_favorite_7d_sum",
    "c_user_author_read_comment_7d_sum",
]


def load_vocabulary(vocab_dir: str, filename: str):
    """Vocabulary file -> list of stripped lines; a missing file is an empty vocabulary
    (dcn.py:154-159)."""
    path = os.path.join(vocab_dir, filename)
    if not os.path.exists(path):
        return []
    with open(path, "r") as f:
        return [line.strip() for line in f]


def table_rows(vocab_dir, field: str, vocab_sizes: Optional[dict] = None) -> int:
    """Embedding rows of a field: len(vocab)+1 (dcn.py:118-126); `vocab_sizes` overrides the
    vocabulary length per field (used for synthetic configs without vocabulary files)."""
    if vocab_sizes is not None and field in vocab_sizes:
        return int(vocab_sizes[field]) + 1
    return len(load_vocabulary(vocab_dir, WECHAT_VOCAB_FILES[field])) + 1


# ---------------------------------------------------------------- per-call random weights (H2)
# The reference re-creates these layers inside forward() from the default CPU generator on
# every call; the draw order below is the reference's construction order.  Each draw is an
# H2Spec: the tensor shapes, a `fill` that makes exactly the reference's generator calls into
# preallocated tensors (nn.Linear.reset_parameters' kaiming_uniform_ then uniform_, or
# cross_layer's xavier_normal_ / zeros_), and a `pack` that returns them in the models' layout.
# Drawing into preallocated views instead of constructing nn.Linear modules gives bit-identical
# values (the same generator calls on the same shapes) without the module overhead, and lets the
# per-call mode draw straight into a pinned staging buffer (H2Stage).

@dataclass
class H2Spec:
    shapes: list
    fill: object
    pack: object


def linear_fill(w: torch.Tensor, b: torch.Tensor):
    """nn.Linear.reset_parameters' draws into preallocated tensors: kaiming_uniform_(a=sqrt(5))
    on the weight, then uniform_(-1/sqrt(fan_in), 1/sqrt(fan_in)) on the bias."""
    nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    fan_in = w.shape[1]
    bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
    nn.init.uniform_(b, -bound, bound)


def cross_spec(dim: int, num_layers: int) -> H2Spec:
    """cross_layer(): w ~ xavier_normal_ on a (d, 1) tensor, b = 0, per layer (dcn.py:37-41)."""
    def fill(v):
        for l in range(num_layers):
            nn.init.xavier_normal_(v[0][l].view(dim, 1))
            nn.init.zeros_(v[1][l].view(dim, 1))
    return H2Spec([(num_layers, dim), (num_layers, dim)], fill, lambda v: (v[0], v[1]))


def din_attention_spec(embedding_dim: int) -> H2Spec:
    """din_attention(): Linear(4H,64), Linear(64,32), Linear(32,1) in order (din.py:61-67)."""
    H = embedding_dim

    def fill(v):
        linear_fill(v[0], v[1])
        linear_fill(v[2], v[3])
        linear_fill(v[4], v[5])
    return H2Spec([(64, 4 * H), (64,), (32, 64), (32,), (1, 32), (1,)], fill, list)


def residual_spec(dim: int, internal_dim: int, num_units: int) -> H2Spec:
    """residual_unit(): Linear(d, I) then Linear(I, d), per unit (deepcrossing.py:37-39)."""
    def fill(v):
        for u in range(num_units):
            linear_fill(v[4 * u], v[4 * u + 1])
            linear_fill(v[4 * u + 2], v[4 * u + 3])
    shapes = [(internal_dim, dim), (internal_dim,), (dim, internal_dim), (dim,)] * num_units
    return H2Spec(shapes, fill, lambda v: [list(v[4 * u:4 * u + 4]) for u in range(num_units)])


def draw_spec(spec: H2Spec):
    """The spec's draws into fresh host tensors."""
    views = [torch.empty(s) for s in spec.shapes]
    spec.fill(views)
    return spec.pack(views)


def draw_cross_layers(dim: int, num_layers: int):
    return draw_spec(cross_spec(dim, num_layers))


def draw_din_attention(embedding_dim: int):
    return draw_spec(din_attention_spec(embedding_dim))


def draw_residual_units(dim: int, internal_dim: int, num_units: int):
    return draw_spec(residual_spec(dim, internal_dim, num_units))


class H2Stage:
    """Per-call draws for a GPU forward: the generator calls write straight into one of two pinned
    host buffers, one asynchronous host-to-device copy per forward moves them into a fresh device
    buffer (stream-ordered before the forward's kernels; the caching allocator keeps it alive for
    them), and the device views are returned in the model's layout.  A buffer is reused only after
    the copy that read it has completed (its event)."""

    def __init__(self):
        self._host = [None, None]
        self._events = [None, None]
        self._turn = 0

    def draw(self, spec: H2Spec, device):
        sizes = [math.prod(s) for s in spec.shapes]
        n = sum(sizes)
        i = self._turn
        self._turn ^= 1
        ev = self._events[i]
        if ev is not None:
            ev.synchronize()
        host = self._host[i]
        if host is None or host.numel() < n:
            host = torch.empty(max(n, 1024), dtype=torch.float32, pin_memory=True)
            self._host[i] = host
        views, off = [], 0
        for s, k in zip(spec.shapes, sizes):
            views.append(host[off:off + k].view(s))
            off += k
        spec.fill(views)
        dev = torch.empty(max(n, 1), dtype=torch.float32, device=device)
        dev[:n].copy_(host[:n], non_blocking=True)
        if ev is None:
            ev = self._events[i] = torch.cuda.Event()  # one event per buffer, re-recorded per use
        ev.record(torch.cuda.current_stream(device))
        out, off = [], 0
        for s, k in zip(spec.shapes, sizes):
            out.append(dev[off:off + k].view(s))
            off += k
        return spec.pack(out)


class InteractionWeights:
    """Holds the H2 weights for one model.  mode 'per_call' redraws them on every forward
    exactly like the reference; 'frozen' draws them once (on the first forward, with the same
    generator calls) and keeps them resident on the device.  `spec` returns the H2Spec of the
    draws (shapes, the reference's generator calls, layout)."""

    MODES = ("per_call", "frozen")

    def __init__(self, mode: str, spec):
        if mode not in self.MODES:
            raise ValueError(f"interaction_weights must be one of {self.MODES}, got {mode!r}")
        self.mode = mode
        self._spec = spec
        self._cached = None
        self._stage = H2Stage()

    def get(self, device):
        if self.mode == "frozen" and self._cached is not None and self._cached[0] == device:
            return self._cached[1]
        if torch.device(device).type == "cuda" and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("per-call interaction weights are drawn on the host each forward and cannot be "
                               "captured in a hipGraph; use interaction_weights='frozen' (or run the forward once "
                               "before capturing)")
        if self.mode == "per_call" and torch.device(device).type == "cuda":
            return self._stage.draw(self._spec(), device)
        dev = _to_device(draw_spec(self._spec()), device)
        if self.mode == "frozen":
            self._cached = (device, dev)
        return dev


def _to_device(obj, device):
    if isinstance(obj, torch.Tensor):
        return obj.to(device).contiguous()
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_device(o, device) for o in obj)
    return obj


# ---------------------------------------------------------------- caches keyed on tensor versions

_GENERATION = [0]


class EngineModule(nn.Module):
    """Base of the drop-in models: any `.to()/.cuda()/.cpu()/.float()` (nn.Module._apply)
    invalidates every derived-tensor cache (folded BatchNorm, packed weights), so a storage that
    lands at a previously used address can never revive a stale cache entry."""

    def _apply(self, fn, *args, **kwargs):
        _GENERATION[0] += 1
        return super()._apply(fn, *args, **kwargs)

    def __getstate__(self):
        # the EagerCalls cache holds ctypes argument blocks (raw device pointers): never pickled
        # or deep-copied with the module; a copy builds its own
        state = self.__dict__.copy()
        state.pop("_eager", None)
        return state

    def train(self, mode: bool = True):
        # A mode switch also invalidates every derived cache: replays of a captured train step
        # (hipGraph) update weights and BatchNorm running statistics without bumping tensor
        # versions, and the reference's loop always calls model.eval() before evaluate()
        # (dcn.py:215, din.py:442-446), so the first eval forward after training re-folds.
        _GENERATION[0] += 1
        return super().train(mode)


def _key(tensors):
    return (_GENERATION[0],) + tuple((t.data_ptr(), t._version) if t is not None else None for t in tensors)


# ---------------------------------------------------------------- eager eval forwards

def tensor_sig(t: torch.Tensor):
    """What a marshalled launch binds of an input tensor: its storage address, dtype, shape and
    strides (not its contents — the kernels read those at launch time)."""
    return (t.data_ptr(), t.dtype, t.shape, t.stride())


class EagerCalls:
    """Marshalled C-ABI calls of one model's eval forward, reused across eager forwards.

    The reference's evaluate() / predict loops call the model eagerly once per batch
    (dcn.py:214-239); rebuilding every ctypes segment, layer and epilogue struct per call cost more
    host time than the forward's kernels.  An entry is keyed on the input tensors' addresses,
    dtypes, shapes and strides, on every parameter / buffer (address, version), on the module
    generation (bumped by .to() / .train() / .eval()) and on the stream, so any change of what a
    launch binds builds a new entry; the output tensors are allocated fresh on every call and
    patched into the cached argument blocks (callers may keep the previous outputs).  Steady-state
    loops alternate between a few input buffers of the caching allocator: a handful of entries."""

    def __init__(self, size: int = 4):
        self._d = {}
        self._size = size
        self._watch = None  # (generation, [parameters and buffers])

    def watched(self, module: nn.Module):
        if self._watch is None or self._watch[0] != _GENERATION[0]:
            self._watch = (_GENERATION[0], [t for t in module.parameters()] + [t for t in module.buffers()])
        return self._watch[1]

    def key(self, module: nn.Module, inputs, stream: int, extra=()):
        ws = self.watched(module)
        return ((_GENERATION[0], stream) + tuple(map(tensor_sig, inputs))
                + tuple((t.data_ptr(), t._version) for t in ws) + tuple(extra))

    def get(self, key):
        return self._d.get(key)

    def put(self, key, entry):
        if len(self._d) >= self._size:
            self._d.pop(next(iter(self._d)))
        self._d[key] = entry
        return entry


class FoldedBN:
    """BatchNorm1d (eval) as a per-channel affine z*scale + shift, recomputed on the device only
    when a running stat or affine parameter changed."""

    def __init__(self):
        self._key = None
        self._val = None

    def __call__(self, bn: nn.BatchNorm1d):
        t = (bn.running_mean, bn.running_var, bn.weight, bn.bias)
        k = _key(t) + (bn.eps,)
        if k != self._key:
            dev = bn.running_mean.device
            scale = torch.empty(bn.num_features, device=dev, dtype=torch.float32)
            shift = torch.empty_like(scale)
            ops.bn_fold(bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.eps, scale, shift)
            self._key, self._val = k, (scale, shift)
        return self._val


class Packed:
    """Row-concatenation of parameters (e.g. [W_q; W_k]) cached on parameter versions."""

    def __init__(self):
        self._key = None
        self._val = None

    def __call__(self, *tensors):
        k = _key(tensors)
        if k != self._key:
            self._key, self._val = k, torch.cat([t.detach() for t in tensors], 0).contiguous()
        return self._val


class PackedFMTable:
    """One field's [V, D] second-order and [V, 1] first-order embedding weights as one packed
    [V, pad4(D+1)] table (rk_fm_pack_table), rebuilt only when either weight's storage or version
    changes or the module moved / switched mode (_GENERATION)."""

    def __init__(self):
        self._key = None
        self._val = None

    def __call__(self, second: torch.Tensor, first: torch.Tensor) -> torch.Tensor:
        k = _key((second, first)) + (tuple(second.shape),)
        if k != self._key:
            self._val = None  # release the stale image before allocating its replacement
            D = second.shape[1]
            self._val = ops.fm_pack_table(second.detach(), first.detach(), (D + 1 + 3) // 4 * 4)
            self._key = k
        return self._val


_CONST = {}


def const(device, value: float):
    key = (str(device), value)
    if key not in _CONST:
        _CONST[key] = torch.full((1,), value, device=device, dtype=torch.float32)
    return _CONST[key]


# ---------------------------------------------------------------- fused MLP tail

@dataclass
class Layer:
    linear: nn.Linear
    pre_bn: Optional[nn.BatchNorm1d] = None   # BatchNorm before the activation
    act: str = "none"
    slope: float = 0.0
    act_module: Optional[nn.Module] = None    # Dice (alpha + its BatchNorm1d(affine=False)) / PReLU
    post_bn: Optional[nn.BatchNorm1d] = None  # BatchNorm after the activation (DIN)
    fold_pre: Optional[FoldedBN] = None
    fold_dice: Optional[FoldedBN] = None
    fold_post: Optional[FoldedBN] = None

    def __post_init__(self):
        self.fold_pre, self.fold_dice, self.fold_post = FoldedBN(), FoldedBN(), FoldedBN()

    def epilogue_kwargs(self):
        kw = dict(bias=self.linear.bias, act=self.act, slope=self.slope)
        if self.pre_bn is not None:
            kw["pre_scale"], kw["pre_shift"] = self.fold_pre(self.pre_bn)
        if self.act == "dice":
            kw["act_scale"], kw["act_shift"] = self.fold_dice(self.act_module.bn)
            kw["act_alpha"], kw["act_alpha_len"] = self.act_module.alpha, self.act_module.alpha.numel()
        elif self.act == "prelu":
            kw["act_alpha"], kw["act_alpha_len"] = self.act_module.weight, self.act_module.weight.numel()
        if self.post_bn is not None:
            kw["post_scale"], kw["post_shift"] = self.fold_post(self.post_bn)
        return kw


EAGER_CACHE = True  # eval forwards reuse their marshalled launches (EagerCalls); False: rebuild per call
FUSED_MLP = True  # one rk_mlp_forward launch per tail when the widths fit (see fused_mlp_fits)
FUSED_GATHER_MLP = True  # DeepCrossing: the row gather inside that launch (rk_mlp_forward_gather)
FUSED_DIN = True  # DIN: gather + attention + fcn tail + head in one rk_din_forward launch
FUSED_BST = True  # BST: all transformer blocks + pooling in one rk_bst_forward_blocks launch
FUSED_BST_FWD = True  # BST at d_model 16: row gather + blocks + pooling + DNN tail in one rk_bst_small_forward
# A first layer this wide runs as its own 2D-tiled GEMM (rk_linear_tiled) before the fused tail:
# in the 16-row fused kernel every CU would stream the whole weight (DeepFM 960 -> 512: 2 MB)
TILED_FIRST_MIN_K = 512
TILED_FIRST_MIN_ROWS = 2048


def _pad64(v: int) -> int:
    return (v + 63) // 64 * 64


_CUS = {}


def _num_cus(device) -> int:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _CUS:
        _CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return _CUS[idx]


def fused_mlp_fits(k0: int, widths) -> bool:
    if len(widths) == 0 or len(widths) > 8 or max(widths) > 512 or _pad64(k0) > 1024:
        return False
    need0 = max([_pad64(k0)] + [_pad64(n) for i, n in enumerate(widths) if i % 2 == 1])
    need1 = max([64] + [_pad64(n) for i, n in enumerate(widths) if i % 2 == 0])
    return 16 * (need0 + 8 + need1 + 8) * 4 <= 160 * 1024  # rows padded by kMlpLdPad (mlp_core.h)


class PackedWeights:
    """Packed weight images (rk_mlp_pack_weight, or the `pack` given), held weakly per weight
    tensor object and rebuilt when its storage or version changes (load_state_dict, .to(),
    optimizer steps).  Keying on the object — not the address — keeps a freed model's packed
    image from being served to a new tensor that reuses its memory.  After an optimizer step the
    image is rewritten in place, on the current stream, unless a prepared forward (DIN / DCN /
    DeepFM .prepare) pinned it: such a plan keeps the image it was prepared with (it binds the
    weights of that moment; prepare again after changing them), and its launches on other streams
    never see a half-rewritten image."""

    def __init__(self, pack=None):
        self._d = {}  # id(tensor) -> (weakref, key, packed, pinned); the weakref callback drops the entry
        self._pack = pack or (lambda w, out=None: ops.pack_mlp_weight(w, out=out))

    def __call__(self, w: torch.Tensor) -> torch.Tensor:
        key = (_GENERATION[0], w.data_ptr(), w._version, tuple(w.shape), w.device)
        hit = self._d.get(id(w))
        if hit is None or hit[0]() is not w or hit[1] != key:
            d, i = self._d, id(w)
            if hit is not None and hit[0]() is w and hit[1][:2] == key[:2] and hit[1][3:] == key[3:] \
                    and not hit[3] and not torch.cuda.is_current_stream_capturing():
                # only the version moved (an optimizer step): rewrite the image in place, on the
                # stream, behind every launch already reading it
                hit = (hit[0], key, self._pack(w, out=hit[2]), False)
            else:
                ref = weakref.ref(w, lambda _r, d=d, i=i: d.pop(i, None) if d.get(i, (None,))[0] is _r else None)
                hit = (ref, key, self._pack(w), False)
            self._d[i] = hit
        return hit[2]

    def pin(self, w: torch.Tensor) -> torch.Tensor:
        """The current image of `w`, never rewritten in place from now on (a later version of `w`
        gets a fresh image)."""
        img = self(w)
        h = self._d[id(w)]
        self._d[id(w)] = (h[0], h[1], h[2], True)
        return img


PACKED = PackedWeights()
BST_PACKED = PackedWeights(lambda w, out=None: ops.pack_bst_weight(w, out=out))  # bst_block_kernel's projections


def empty_rows(device, n: int, shape=(0, 1)):
    """The outputs of an eval forward over an empty batch: n empty float32 tensors of the model's
    output shape.  The reference's torch ops return empty outputs there; the engine launches no
    kernel (an empty tensor's data pointer may be null, which the C ABI rejects)."""
    return tuple(torch.empty(shape, device=device, dtype=torch.float32) for _ in range(n))


def tiled_layer(K: int, B: int, device, ml) -> bool:
    """Whether a K-wide layer of the fused path runs as its own 2D-tiled GEMM (rk_linear_tiled,
    64 x 128 tiles): wide enough, and that grid still fills the GPU (DeepFM: 960 -> 512 yes,
    512 -> 256 no: 128 tiles measured slower than the fused kernel)."""
    return bool(TILED_FIRST_MIN_K and K >= TILED_FIRST_MIN_K and B >= TILED_FIRST_MIN_ROWS and ml.residual == 0
                and ((B + 63) // 64) * ((_pad64(ml.n) + 127) // 128) >= _num_cus(device))


def run_tail(x: torch.Tensor, layers, head: nn.Linear, head_kwargs: dict, logit: torch.Tensor,
             prob: torch.Tensor):
    """Runs the hidden layers and the final Linear(N, 1) + sigmoid.  Normally one fused
    rk_mlp_forward launch; otherwise per-layer rk_linear with the head fused into the last
    layer's epilogue when its width fits one workgroup (N <= 256)."""
    h = x
    B = x.shape[0]
    dev = x.device
    head_w = head.weight
    if FUSED_MLP and fused_mlp_fits(x.shape[1], [l.linear.out_features for l in layers]):
        mls = [ops.make_mlp_layer(l.linear.weight, PACKED(l.linear.weight), **l.epilogue_kwargs()) for l in layers]
        ep = ops.make_epilogue(head_w=head_w, head_b=head.bias, head_logit=logit, head_prob=prob, **head_kwargs)
        # leading wide layers as 2D-tiled GEMMs (tiled_layer), the rest fused
        i = 0
        while i < len(mls) - 1 and tiled_layer(h.shape[1], B, dev, mls[i]):
            y = torch.empty(B, layers[i].linear.out_features, device=dev, dtype=torch.float32)
            ops.linear_tiled(h, mls[i], y)
            h, i = y, i + 1
        ops.mlp_forward(h, mls[i:], ep)
        return
    for i, layer in enumerate(layers):
        last = i == len(layers) - 1
        lin = layer.linear
        kw = layer.epilogue_kwargs()
        if last and lin.out_features <= 256:
            ep = ops.make_epilogue(head_w=head_w, head_b=head.bias, head_logit=logit, head_prob=prob,
                                   **head_kwargs, **kw)
            ops.linear(h, lin.weight, None, epilogue=ep)
            return
        y = torch.empty(B, lin.out_features, device=dev, dtype=torch.float32)
        ops.linear(h, lin.weight, y, epilogue=ops.make_epilogue(**kw))
        h = y
    # head on its own: z = h . w + b as an N=1 GEMM, then the unit head epilogue
    ep = ops.make_epilogue(bias=head.bias, head_w=const(dev, 1.0), head_b=const(dev, 0.0), head_logit=logit,
                           head_prob=prob, **head_kwargs)
    ops.linear(h, head_w, None, epilogue=ep)


def tail_launches(x: torch.Tensor, layers, head: nn.Linear, head_kwargs: dict):
    """run_tail's fused path as a reusable launch list for EagerCalls: [(C function name, argument
    list)] with the stream slot last (None), the head epilogue (its output pointers — head_logit,
    head_prob, head_aux, fm1 / fm2 — are patched per call) and the objects the argument blocks
    point into.  None when run_tail would not take the fused path."""
    B, dev = x.shape[0], x.device
    if not (FUSED_MLP and fused_mlp_fits(x.shape[1], [l.linear.out_features for l in layers])):
        return None
    packed = [PACKED(l.linear.weight) for l in layers]
    mls = [ops.make_mlp_layer(l.linear.weight, pk, **l.epilogue_kwargs()) for l, pk in zip(layers, packed)]
    ep = ops.make_epilogue(head_w=head.weight, head_b=head.bias, **head_kwargs)
    launches, keep = [], [packed, mls]
    h, i = x, 0
    while i < len(mls) - 1 and tiled_layer(h.shape[1], B, dev, mls[i]):
        y = torch.empty(B, layers[i].linear.out_features, device=dev, dtype=torch.float32)
        launches.append(("rk_linear_tiled", [h.data_ptr(), h.stride(0), B, h.shape[1], ops.ctypes.byref(mls[i]),
                                             y.data_ptr(), y.stride(0), None]))
        keep.append(y)
        h, i = y, i + 1
    arr = (ops._lib.MlpLayer * max(1, len(mls) - i))(*mls[i:])
    keep.append(arr)
    launches.append(("rk_mlp_forward", [h.data_ptr(), h.stride(0), B, h.shape[1], arr, len(mls) - i,
                                        ops.ctypes.byref(ep), None, 0, None]))
    return launches, ep, keep


def run_launches(launches, stream: int):
    lib = ops._lib.load()
    for name, args in launches:
        args[-1] = stream
        ops.check(getattr(lib, name)(*args), name)


def check_eval(module: nn.Module):
    if module.training:
        raise NotImplementedError(
            f"{type(module).__name__}: the rankops engine implements the eval-mode forward "
            f"(BatchNorm running stats, Dropout identity); call .eval() first. "
            f"Training (backward) is the next row of the build plan (DESIGN.md).")


def sqrt_f32(x: float) -> float:
    return float(torch.tensor(math.sqrt(x), dtype=torch.float32))
