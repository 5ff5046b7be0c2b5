"""Host input path: raw wechat rows -> the model's forward arguments on the GPU.

Replaces the reference's per-row `WechatDataset.__getitem__` (pandas `iloc` + Python dict
lookups, dcn.py:94-111; din.py:131-173; bst.py:130-159; deepfm.py:56-70; afm.py:46-62;
deepcrossing.py:86-104) and its collate (`din_collate_fn`, din.py:175-222; the default collate
elsewhere) with column-wise bucketing (`include/rankops_io.h`) of Apache Arrow string columns:
on the GPU (default: the raw string bytes travel in the batch's ONE pinned host-to-device copy
and `rk_bucketize*_device` hash them against device copies of the vocabularies) or by C++ host
threads writing the int64 rows into that pinned buffer.  Semantics are the reference's bit for bit (hazard H1): the position of
the stripped line in the vocabulary file (last duplicate wins), 0 for unknown or null values,
DIN histories split on ',' ('' is one item) and zero-padded to the batch maximum, BST's
one-item sequence padded to max_seq_length.  tests/test_loader.py checks every case against
the pure-Python restatement in oracle/bucketing.py.

    vocabs = wechat_vocabularies(vocab_dir)                 # once
    asm = BatchAssembler("din", vocabs, device="cuda")
    dense, category, sequence, target = asm(arrow_table)    # per batch (pyarrow.Table or dict)
    prob, logit, l2 = din_model(dense, category, sequence, target)
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib

DENSE_FEATURES = (
    "videoplayseconds", "u_read_comment_7d_sum", "u_like_7d_sum", "u_click_avatar_7d_sum",
    "u_forward_7d_sum", "u_comment_7d_sum", "u_follow_7d_sum", "u_favorite_7d_sum",
    "i_read_comment_7d_sum", "i_like_7d_sum", "i_click_avatar_7d_sum", "i_forward_7d_sum",
    "i_comment_7d_sum", "i_follow_7d_sum", "i_favorite_7d_sum", "c_user_author_read_comment_7d_sum")
VOCAB_FILES = {"userid": "userid.txt", "feedid": "feedid.txt", "device": "device.txt",
               "authorid": "authorid.txt", "bgm_song_id": "bgm_song_id.txt",
               "bgm_singer_id": "bgm_singer_id.txt", "manual_tag_list": "manual_tag_id.txt"}
DIN_SEQ = "his_read_comment_7d_seq"
CATEGORY = {
    "dcn": ("userid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"),
    "deepcrossing": ("userid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"),
    "din": ("userid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"),
    "bst": ("userid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"),
    "deepfm": ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id"),
    "afm": ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"),
}


class Vocabulary:
    """One vocabulary file, bucketing in C++ (rk_vocab_*).  `len(v)` is len(vocab); embedding
    tables have len(v) + 1 rows.  skip_empty_lines=True is AFM's variant (afm.py:33-35)."""

    def __init__(self, path=None, *, text: bytes = None, skip_empty_lines=False):
        lib = _lib.load()
        if (path is None) == (text is None):
            raise ValueError("Vocabulary: give exactly one of path / text")
        if path is not None:
            h = lib.rk_vocab_load(os.fsencode(path), 1 if skip_empty_lines else 0)
        else:
            h = lib.rk_vocab_parse(bytes(text), len(text), 1 if skip_empty_lines else 0)
        if not h:
            raise _lib.RankOpsError(f"Vocabulary: {_lib.last_error()}")
        self._h = h
        self.path = path
        self.skip_empty_lines = skip_empty_lines

    def __len__(self):
        return int(_lib.load().rk_vocab_size(self._h))

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _lib._lib is not None:
            _lib._lib.rk_vocab_free(h)

    def lookup(self, column, out: np.ndarray = None, threads: int = 0) -> np.ndarray:
        """int64 row of every value of `column` (0 for unknown / null / non-string values)."""
        chunks = _arrow_chunks(column)
        n = sum(len(c) for c in chunks)
        if out is None:
            out = np.empty(n, dtype=np.int64)
        _bucketize_into(self, chunks, out.ctypes.data, 1, threads)
        return out

    def to_device(self, device="cuda"):
        """(slots, arena, mask): the hash table copied to `device` once (rk_vocab_export) for
        the *_device lookups; cached per device."""
        dev = torch.device(device)
        key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
        cache = self.__dict__.setdefault("_device_tables", {})
        if key not in cache:
            lib = _lib.load()
            sb, ab, mask = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_uint64()
            _lib.check(lib.rk_vocab_export_size(self._h, ctypes.byref(sb), ctypes.byref(ab), ctypes.byref(mask)),
                       "rk_vocab_export_size")
            slots = torch.empty(sb.value, dtype=torch.uint8)
            arena = torch.empty(ab.value, dtype=torch.uint8)
            _lib.check(lib.rk_vocab_export(self._h, slots.data_ptr(), arena.data_ptr()), "rk_vocab_export")
            cache[key] = (slots.to(dev), arena.to(dev), int(mask.value))
        return cache[key]

    def lookup_device(self, column, device="cuda") -> torch.Tensor:
        """lookup() on the GPU (rk_bucketize_device): the column's raw strings are copied to
        `device` and looked up there.  Returns an int64 device tensor."""
        return _device_lookup(self, _arrow_chunks(column), torch.device(device), None, ",")

    def lookup_sequences_device(self, column, T: int = None, sep=",", device="cuda", null_history="raise"):
        """lookup_sequences() on the GPU (rk_bucketize_sequences_device)."""
        chunks = _arrow_chunks(column)
        _check_null_history(chunks, null_history, "lookup_sequences_device")
        if T is None:
            T = _max_items(chunks, sep, 0)
        return _device_lookup(self, chunks, torch.device(device), T, sep)

    def lookup_sequences(self, column, T: int = None, sep=",", threads: int = 0, null_history="raise"):
        """(idx [n, T] int64 zero padded, lengths [n]) of sep-separated histories; T defaults to
        the longest row (din_collate_fn).  A null value raises TypeError as the reference's
        Dataset does (din.py:147-151) unless null_history="empty" (length 0)."""
        chunks = _arrow_chunks(column)
        _check_null_history(chunks, null_history, "lookup_sequences")
        n = sum(len(c) for c in chunks)
        if T is None:
            T = _max_items(chunks, sep, threads)
        out = np.empty((n, T), dtype=np.int64)
        lens = np.empty(n, dtype=np.int64)
        _sequences_into(self, chunks, sep, T, out.ctypes.data, T, lens.ctypes.data, threads)
        return out, lens


def label_encode(column, vocab: "Vocabulary | None", threads: int = 0) -> np.ndarray:
    """FwFM's dataset-level LabelEncoder bucketing of one whole column (fwfm.py:29-31,48-67):
    null and "None" are NaN; NaN and out-of-vocabulary values take the index of the column's
    mode (most frequent non-NaN value, ties -> smallest string; 'unknown' when every value is
    NaN); index = position of the last occurrence of the stripped line in the vocabulary file
    (LabelEncoder with classes_ = the file's lines, no empty-line skipping, no +1).  Raises
    ValueError where the reference's LabelEncoder.transform raises (the mode itself is not in
    the vocabulary).  An empty / missing vocabulary parses the values as Python int()
    (`.fillna(0).astype(int)`, ASCII digits only).  rk_label_encode, C++ threads."""
    pa = _pa()
    lib = _lib.load()
    if isinstance(column, pa.ChunkedArray):
        arr = pa.concat_arrays(column.chunks) if column.num_chunks != 1 else column.chunk(0)
    elif isinstance(column, pa.Array):
        arr = column
    else:
        if hasattr(column, "to_numpy") and not isinstance(column, np.ndarray):  # pandas Series
            column = column.to_numpy(dtype=object)
        arr = pa.array(list(column))
    if pa.types.is_dictionary(arr.type):
        arr = arr.dictionary_decode()
    if pa.types.is_integer(arr.type) and arr.null_count == 0:
        arr = arr.cast(pa.string())  # .astype(str) of an int column: str(int)
    if not (pa.types.is_string(arr.type) or pa.types.is_large_string(arr.type) or pa.types.is_null(arr.type)):
        raise TypeError(f"label_encode: column type {arr.type} is not supported (string, or integer without nulls)")
    if pa.types.is_null(arr.type):
        arr = arr.cast(pa.string())
    n = len(arr)
    out = np.empty(n, dtype=np.int64)
    if n == 0:
        return out
    d, o, bits, v, vo = _buffers(arr)
    mode = ctypes.c_int64()
    rc = lib.rk_label_encode(vocab._h if vocab is not None and len(vocab) else None, d, o, bits, v, vo, n,
                             out.ctypes.data, ctypes.byref(mode), threads)
    if rc != 0:
        raise ValueError(_lib.last_error())
    return out


def wechat_vocabularies(vocab_dir, fields=tuple(VOCAB_FILES), skip_empty_lines=False):
    """{field: Vocabulary} with the reference's field -> file mapping (manual_tag_list reads
    manual_tag_id.txt, dcn.py:66).  A missing file gives an empty vocabulary (dcn.py:86-87)."""
    out = {}
    for f in fields:
        path = os.path.join(vocab_dir, VOCAB_FILES[f])
        out[f] = Vocabulary(path, skip_empty_lines=skip_empty_lines) if os.path.exists(path) else \
            Vocabulary(text=b"", skip_empty_lines=skip_empty_lines)
    return out


# ---------------------------------------------------------------- Arrow plumbing

def _pa():
    import pyarrow as pa
    return pa


def _arrow_chunks(column):
    """Column -> list of pyarrow string / large_string Arrays (None for non-string columns, which
    the reference never matches against its str-keyed dicts)."""
    pa = _pa()
    if isinstance(column, pa.ChunkedArray):
        chunks = list(column.chunks)
    elif isinstance(column, pa.Array):
        chunks = [column]
    else:
        if hasattr(column, "to_numpy") and not isinstance(column, np.ndarray):  # pandas Series
            column = column.to_numpy(dtype=object)
        vals = list(column)
        if all(v is None or isinstance(v, str) for v in vals):
            chunks = [pa.array(vals, type=pa.string())]
        else:  # mixed / non-str values: only str values can match (dict keys are str)
            chunks = [pa.array([v if isinstance(v, str) else None for v in vals], type=pa.string())]
    out = []
    for c in chunks:
        if pa.types.is_dictionary(c.type):
            c = c.dictionary_decode()
        if pa.types.is_string(c.type) or pa.types.is_large_string(c.type):
            out.append(c)
        else:
            out.append(_NonString(len(c)))
    return out


class _NonString:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


def _buffers(arr):
    """(data ptr, offsets ptr at the slice start, offset bits, validity ptr, validity bit offset)."""
    pa = _pa()
    bits = 64 if pa.types.is_large_string(arr.type) else 32
    validity, offsets, data = arr.buffers()
    off_ptr = offsets.address + arr.offset * (bits // 8)
    data_ptr = data.address if data is not None and data.size > 0 else off_ptr  # any non-null pointer
    valid_ptr = validity.address if (validity is not None and arr.null_count > 0) else None
    return data_ptr, off_ptr, bits, valid_ptr, arr.offset


def _bucketize_into(vocab, chunks, out_ptr, stride, threads):
    lib = _lib.load()
    pos = 0
    for c in chunks:
        n = len(c)
        dst = out_ptr + pos * stride * 8
        if isinstance(c, _NonString):
            ctypes.memset(dst, 0, n * 8) if stride == 1 else [ctypes.memset(dst + i * stride * 8, 0, 8)
                                                             for i in range(n)]
        elif n:
            d, o, bits, v, vo = _buffers(c)
            _lib.check(lib.rk_bucketize(vocab._h, d, o, bits, v, vo, n, dst, stride, threads), "rk_bucketize")
        pos += n


def _max_items(chunks, sep, threads):
    lib = _lib.load()
    m = 0
    for c in chunks:
        if isinstance(c, _NonString) or not len(c):
            continue
        lens = np.empty(len(c), dtype=np.int64)
        mx = ctypes.c_int64(0)
        d, o, bits, v, vo = _buffers(c)
        _lib.check(lib.rk_sequence_lengths(d, o, bits, v, vo, len(c), sep.encode(), lens.ctypes.data,
                                           ctypes.byref(mx), threads), "rk_sequence_lengths")
        m = max(m, int(mx.value))
    return m


def _sequences_into(vocab, chunks, sep, T, out_ptr, ld, len_ptr, threads):
    lib = _lib.load()
    pos = 0
    for c in chunks:
        n = len(c)
        if isinstance(c, _NonString):  # not a str: the reference iterates it; only str items are rejected
            raise TypeError("rankops.loader: a sequence column must hold strings")
        if n:
            d, o, bits, v, vo = _buffers(c)
            _lib.check(lib.rk_bucketize_sequences(vocab._h, d, o, bits, v, vo, n, sep.encode(), T,
                                                  out_ptr + pos * ld * 8, ld, len_ptr + pos * 8, threads),
                       "rk_bucketize_sequences")
        pos += n


def _stage_chunk(c):
    """Host copies (offsets rebased to 0, data, validity bytes, bit offset) of one Arrow chunk."""
    pa = _pa()
    n = len(c)
    bits = 64 if pa.types.is_large_string(c.type) else 32
    validity, offsets, data = c.buffers()
    odt = np.int64 if bits == 64 else np.int32
    offs = np.frombuffer(offsets, dtype=odt, count=c.offset + n + 1)[c.offset:]
    lo, hi = int(offs[0]), int(offs[-1])
    raw = np.frombuffer(data, dtype=np.uint8, count=hi)[lo:] if hi > lo else np.zeros(1, np.uint8)
    vb = None
    if c.null_count > 0:
        b0 = c.offset >> 3
        nb = (c.offset + n + 7) // 8 - b0
        vb = np.frombuffer(validity, dtype=np.uint8, count=b0 + nb)[b0:]
    return bits, (offs - offs.dtype.type(lo)), raw, vb, c.offset & 7


def _device_lookup(vocab, chunks, dev, T, sep):
    lib = _lib.load()
    n = sum(len(c) for c in chunks)
    if T is None:
        out = torch.zeros(max(n, 1), dtype=torch.int64, device=dev)[:n]
        lens = None
    else:
        out = torch.zeros(n, T, dtype=torch.int64, device=dev)
        lens = torch.zeros(n, dtype=torch.int64, device=dev)
    slots, arena, mask = vocab.to_device(dev)
    stream = _lib.raw_stream(dev)
    keep = []
    r0 = 0
    for c in chunks:
        if isinstance(c, _NonString):
            if T is not None:
                raise TypeError("rankops.loader: a sequence column must hold strings")
            r0 += len(c)
            continue
        if len(c) == 0:
            continue
        bits, offs, raw, vb, bit0 = _stage_chunk(c)
        d_offs = torch.from_numpy(np.ascontiguousarray(offs)).to(dev)
        d_raw = torch.from_numpy(np.ascontiguousarray(raw)).to(dev)
        d_vb = torch.from_numpy(np.ascontiguousarray(vb)).to(dev) if vb is not None else None
        keep += [d_offs, d_raw, d_vb]
        args = (slots.data_ptr(), mask, arena.data_ptr(), d_raw.data_ptr(), d_offs.data_ptr(), bits,
                d_vb.data_ptr() if d_vb is not None else None, bit0 if d_vb is not None else 0, len(c))
        if T is None:
            _lib.check(lib.rk_bucketize_device(*args, out.data_ptr() + r0 * 8, 1, stream), "rk_bucketize_device")
        else:
            _lib.check(lib.rk_bucketize_sequences_device(*args, sep.encode(), T, out.data_ptr() + r0 * T * 8, T,
                                                         lens.data_ptr() + r0 * 8, stream),
                       "rk_bucketize_sequences_device")
        r0 += len(c)
    torch.cuda.current_stream(dev).synchronize()  # the staged inputs are freed on return
    return out if T is None else (out, lens)


def _column(table, name):
    pa = _pa()
    if isinstance(table, pa.Table):
        return table.column(name) if name in table.column_names else None
    return table.get(name)


def _num_rows(table):
    pa = _pa()
    if isinstance(table, pa.Table):
        return table.num_rows
    for v in table.values():
        return len(v)
    return 0


def _dense_into(table, name, out: np.ndarray):
    """row.get(f, 0.0) -> float32 (dcn.py:97): float64 values rounded to float32, nulls NaN."""
    col = _column(table, name)
    if col is None:
        out[...] = 0.0
        return
    pa = _pa()
    if isinstance(col, (pa.Array, pa.ChunkedArray)):
        col = col.to_numpy(zero_copy_only=False)
    out[...] = np.asarray(col, dtype=np.float64).astype(np.float32)


# ---------------------------------------------------------------- batch assembly

NULL_HISTORY = ("raise", "empty")


def _check_null_history(chunks, policy: str, what: str):
    """A null history cell.  The reference's DIN Dataset reads it with row.get(col, []), which
    returns the null (None / NaN) for a present column, and then iterates it: TypeError
    (din.py:147-151).  policy "raise" (default) does the same; "empty" reads it as an empty history
    (length 0), which only a row WITHOUT the column gets in the reference."""
    if policy not in NULL_HISTORY:
        raise ValueError(f"{what}: null_history must be one of {NULL_HISTORY}, got {policy!r}")
    if policy == "raise" and chunks is not None:
        for c in chunks:
            if not isinstance(c, _NonString) and c.null_count > 0:
                raise TypeError(f"{what}: null history value ('NoneType' object is not iterable, as the "
                                "reference's DIN Dataset raises at din.py:147-151); pass null_history='empty' "
                                "to read nulls as empty histories")


class BatchAssembler:
    """Builds one model's forward arguments for a batch of raw rows.

    bucketing="device" (default on a GPU): the batch's raw Arrow string buffers (rebased per
    column) and its float32 dense block are packed into ONE pinned host buffer, sent in one
    asynchronous host-to-device copy, and rk_bucketize_device / rk_bucketize_sequences_device
    turn the strings into int64 rows in HBM against the vocabularies' device tables.
    bucketing="host": the int64 rows are produced by the C++ host lookups straight into the
    pinned buffer, then copied the same way.  The pinned buffers are double-buffered (the next
    batch is packed while the previous copy may still be in flight); the returned tensors are
    views of device buffers.  With device="cpu" the host path returns host tensors."""

    def __init__(self, model: str, vocabs: dict, device="cuda", max_seq_length=50, threads: int = 0,
                 bucketing: str = None, null_history: str = "raise"):
        if model not in CATEGORY:
            raise ValueError(f"BatchAssembler: unknown model {model!r}")
        _check_null_history(None, null_history, "BatchAssembler")
        self.null_history = null_history  # DIN: a null history raises TypeError (din.py:147-151) or reads as []
        bucketing = bucketing or ("device" if torch.device(device).type == "cuda" else "host")
        if bucketing not in ("host", "device"):
            raise ValueError(f"BatchAssembler: bucketing must be 'host' or 'device', got {bucketing!r}")
        if bucketing == "device" and torch.device(device).type != "cuda":
            raise ValueError("BatchAssembler: device bucketing needs a GPU device")
        self.bucketing = bucketing
        self.model = model
        self.vocabs = vocabs
        self.device = torch.device(device)
        self.max_seq_length = max_seq_length
        self.threads = threads
        self._pinned = [None, None]
        self._events = [None, None]
        self._turn = 0

    def _host_buffer(self, nbytes):
        i = self._turn
        self._turn ^= 1
        if self._events[i] is not None:
            self._events[i].synchronize()  # its previous copy must have left the buffer
        buf = self._pinned[i]
        if buf is None or buf.numel() < nbytes:
            pin = self.device.type == "cuda"
            buf = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8, pin_memory=pin)
            self._pinned[i] = buf
        return i, buf

    def __call__(self, table):
        if self.bucketing == "device":
            return self._call_device(table)
        m = self.model
        B = _num_rows(table)
        cats = CATEGORY[m]
        seq_T = 0
        hist = None
        if m == "din":
            hist = _arrow_chunks(_column(table, DIN_SEQ)) if _column(table, DIN_SEQ) is not None else None
            _check_null_history(hist, self.null_history, "BatchAssembler")
            seq_T = _max_items(hist, ",", self.threads) if hist is not None else 0
        elif m == "bst":
            seq_T = self.max_seq_length
        # int64 region: categories [F][B] | target [B] | seq [B][T] | lengths [B];  float32 dense [16][B] or [B][16]
        n_i64 = len(cats) * B + (B if m == "din" else 0) + B * seq_T + (B if m in ("din", "bst") else 0)
        n_f32 = 0 if m == "deepfm" else 16 * B
        nbytes = n_i64 * 8 + n_f32 * 4
        slot, buf = self._host_buffer(nbytes)
        base = buf.data_ptr()
        host_i64 = buf[:n_i64 * 8].view(torch.int64).numpy()
        host_f32 = buf[n_i64 * 8:nbytes].view(torch.float32).numpy()

        p = 0
        cat_off = {}
        for c in cats:
            cat_off[c] = p
            col = _column(table, c)
            vocab = self.vocabs.get(c) if not (m == "afm" and c == "manual_tag_list") else None
            if col is None or vocab is None:
                host_i64[p:p + B] = 0  # no column / AFM's missing manual_tag_list.txt (afm.py:31-36)
            else:
                _bucketize_into(vocab, _arrow_chunks(col), base + p * 8, 1, self.threads)
            p += B
        tgt_off = seq_off = len_off = None
        if m == "din":
            tgt_off = p
            col = _column(table, "feedid")
            if col is None:
                host_i64[p:p + B] = 0
            else:
                _bucketize_into(self.vocabs["feedid"], _arrow_chunks(col), base + p * 8, 1, self.threads)
            p += B
            seq_off, len_off = p, p + B * seq_T
            if hist is None:  # row.get(col, []) on a missing column
                host_i64[len_off:len_off + B] = 0
            else:
                _sequences_into(self.vocabs["feedid"], hist, ",", seq_T, base + seq_off * 8, seq_T,
                                base + len_off * 8, self.threads)
            p = len_off + B
        elif m == "bst":
            seq_off, len_off = p, p + B * seq_T
            seq = host_i64[seq_off:len_off].reshape(B, seq_T)
            seq[...] = 0
            col = _column(table, "feedid")
            if seq_T > 0:
                if col is None:  # row.get("feedid", []) -> []: length 0
                    host_i64[len_off:len_off + B] = 0
                else:  # [row['feedid']]: one item (bst.py:142-150)
                    _bucketize_into(self.vocabs["feedid"], _arrow_chunks(col), base + seq_off * 8, seq_T,
                                    self.threads)
                    host_i64[len_off:len_off + B] = 1
            else:
                host_i64[len_off:len_off + B] = 0
            p = len_off + B
        if n_f32:
            dense = host_f32.reshape(16, B) if m == "din" else host_f32.reshape(B, 16)
            for j, f in enumerate(DENSE_FEATURES):
                _dense_into(table, f, dense[j] if m == "din" else dense[:, j])

        if self.device.type == "cuda":
            dev = buf[:nbytes].to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._events[slot] = ev
        else:
            dev = buf[:nbytes].clone()
        i64 = dev[:n_i64 * 8].view(torch.int64)
        f32 = dev[n_i64 * 8:nbytes].view(torch.float32)
        category = {c: i64[cat_off[c]:cat_off[c] + B] for c in cats}
        if m in ("dcn", "deepcrossing"):
            return f32.view(B, 16), category
        if m == "deepfm":
            return (category,)
        if m == "afm":
            return f32.view(B, 16), category
        if m == "bst":
            return (f32.view(B, 16), category, i64[seq_off:len_off].view(B, seq_T),
                    i64[len_off:len_off + B])
        # din
        dense = {f: f32[j * B:(j + 1) * B] for j, f in enumerate(DENSE_FEATURES)}
        sequence = {DIN_SEQ: i64[seq_off:len_off].view(B, seq_T), DIN_SEQ + "_length": i64[len_off:len_off + B]}
        target = {"feedid": i64[tgt_off:tgt_off + B]}
        return dense, category, sequence, target

    # ---------------------------------------------------------------- device bucketing
    def _string_jobs(self, table, B):
        """[(kind, vocab, chunks, ...)] of the string columns this model buckets."""
        m = self.model
        jobs = []
        for c in CATEGORY[m]:
            col = _column(table, c)
            vocab = self.vocabs.get(c) if not (m == "afm" and c == "manual_tag_list") else None
            jobs.append(("cat", c, vocab, None if (col is None or vocab is None) else _arrow_chunks(col)))
        if m == "din":
            col = _column(table, "feedid")
            jobs.append(("target", "feedid", self.vocabs["feedid"], None if col is None else _arrow_chunks(col)))
            hist = _column(table, DIN_SEQ)
            jobs.append(("hist", DIN_SEQ, self.vocabs["feedid"], None if hist is None else _arrow_chunks(hist)))
        elif m == "bst":
            col = _column(table, "feedid")
            jobs.append(("bstseq", "feedid", self.vocabs["feedid"], None if col is None else _arrow_chunks(col)))
        return jobs

    def _call_device(self, table):
        m = self.model
        B = _num_rows(table)
        dev = self.device
        lib = _lib.load()
        stream = _lib.raw_stream(dev)
        jobs = self._string_jobs(table, B)
        seq_T = 0
        for kind, _, _, chunks in jobs:
            if kind == "hist" and chunks is not None:
                if any(isinstance(c, _NonString) for c in chunks):
                    raise TypeError("rankops.loader: a sequence column must hold strings")
                _check_null_history(chunks, self.null_history, "BatchAssembler")
                seq_T = _max_items(chunks, ",", self.threads)
        if m == "bst":
            seq_T = self.max_seq_length
        # staging plan: per string chunk [offsets | validity | data], then the dense block
        plan = []
        nbytes = 0

        def reserve(n):
            nonlocal nbytes
            off = nbytes
            nbytes += (n + 15) // 16 * 16
            return off

        for j, (kind, name, vocab, chunks) in enumerate(jobs):
            if chunks is None:
                continue
            for ci, c in enumerate(chunks):
                if isinstance(c, _NonString) or len(c) == 0:
                    continue
                n = len(c)
                bits = 64 if _pa().types.is_large_string(c.type) else 32
                validity, offsets, data = c.buffers()
                odt = np.int64 if bits == 64 else np.int32
                offs = np.frombuffer(offsets, dtype=odt, count=c.offset + n + 1, offset=0)[c.offset:]
                lo, hi = int(offs[0]), int(offs[-1])
                has_nulls = c.null_count > 0
                plan.append(dict(job=j, chunk=ci, n=n, bits=bits, offs=offs, lo=lo, hi=hi, data=data,
                                 validity=validity if has_nulls else None, bit0=c.offset,
                                 o_off=reserve(offs.nbytes), v_off=reserve((n + 7 + 7) // 8) if has_nulls else None,
                                 d_off=reserve(max(hi - lo, 1))))
        n_f32 = 0 if m == "deepfm" else 16 * B
        f_off = reserve(n_f32 * 4)
        slot, buf = self._host_buffer(nbytes)
        hb = buf.numpy()
        for p in plan:
            o = p["offs"]
            dst = hb[p["o_off"]:p["o_off"] + o.nbytes].view(o.dtype)
            np.subtract(o, o.dtype.type(p["lo"]), out=dst)
            if p["hi"] > p["lo"]:
                hb[p["d_off"]:p["d_off"] + p["hi"] - p["lo"]] = np.frombuffer(p["data"], dtype=np.uint8,
                                                                               count=p["hi"], offset=0)[p["lo"]:]
            if p["validity"] is not None:
                b0 = p["bit0"] >> 3
                nb = (p["bit0"] + p["n"] + 7) // 8 - b0
                hb[p["v_off"]:p["v_off"] + nb] = np.frombuffer(p["validity"], dtype=np.uint8,
                                                               count=b0 + nb, offset=0)[b0:]
        if n_f32:
            dense_h = hb[f_off:f_off + n_f32 * 4].view(np.float32)
            dense_h = dense_h.reshape(16, B) if m == "din" else dense_h.reshape(B, 16)
            for jj, f in enumerate(DENSE_FEATURES):
                _dense_into(table, f, dense_h[jj] if m == "din" else dense_h[:, jj])
        staged = buf[:max(nbytes, 1)].to(dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        self._events[slot] = ev
        sbase = staged.data_ptr()

        # int64 outputs on the device: categories [F][B] | target [B] | seq [B][T] | lengths [B]
        cats = CATEGORY[m]
        n_i64 = len(cats) * B + (B if m == "din" else 0) + B * seq_T + (B if m in ("din", "bst") else 0)
        i64 = torch.zeros(max(n_i64, 1), dtype=torch.int64, device=dev)
        obase = i64.data_ptr()
        out_off = {}
        p_ = 0
        for kind, name, _, _ in jobs:
            if kind in ("cat", "target"):
                out_off[(kind, name)] = p_
                p_ += B
        seq_off = len_off = None
        if m in ("din", "bst"):
            seq_off, len_off = p_, p_ + B * seq_T
        row_of_chunk = {}
        for j, (kind, name, vocab, chunks) in enumerate(jobs):
            if chunks is None:
                continue
            r = 0
            for ci, c in enumerate(chunks):
                row_of_chunk[(j, ci)] = r
                r += len(c)
        for p in plan:
            kind, name, vocab, _ = jobs[p["job"]]
            slots, arena, mask = vocab.to_device(dev)
            r0 = row_of_chunk[(p["job"], p["chunk"])]
            valid = sbase + p["v_off"] if p["v_off"] is not None else None
            bit0 = (p["bit0"] & 7) if p["v_off"] is not None else 0
            args = (slots.data_ptr(), mask, arena.data_ptr(), sbase + p["d_off"], sbase + p["o_off"], p["bits"],
                    valid, bit0, p["n"])
            if kind in ("cat", "target"):
                _lib.check(lib.rk_bucketize_device(*args, obase + (out_off[(kind, name)] + r0) * 8, 1, stream),
                           "rk_bucketize_device")
            elif kind == "bstseq":
                if seq_T > 0:
                    _lib.check(lib.rk_bucketize_device(*args, obase + (seq_off + r0 * seq_T) * 8, seq_T, stream),
                               "rk_bucketize_device")
            else:  # DIN history
                _lib.check(lib.rk_bucketize_sequences_device(*args, b",", seq_T, obase + (seq_off + r0 * seq_T) * 8,
                                                             seq_T, obase + (len_off + r0) * 8, stream),
                           "rk_bucketize_sequences_device")
        if m == "bst":  # [row['feedid']]: one item per row (bst.py:142-150); no column: length 0
            has_col = any(k == "bstseq" and ch is not None for k, _, _, ch in jobs)
            i64[len_off:len_off + B].fill_(1 if (has_col and seq_T > 0) else 0)
        f32 = staged[f_off:f_off + n_f32 * 4].view(torch.float32)
        category = {c: i64[out_off[("cat", c)]:out_off[("cat", c)] + B] for c in cats}
        if m in ("dcn", "deepcrossing", "afm"):
            return f32.view(B, 16), category
        if m == "deepfm":
            return (category,)
        if m == "bst":
            return (f32.view(B, 16), category, i64[seq_off:len_off].view(B, seq_T), i64[len_off:len_off + B])
        dense = {f: f32[jj * B:(jj + 1) * B] for jj, f in enumerate(DENSE_FEATURES)}
        sequence = {DIN_SEQ: i64[seq_off:len_off].view(B, seq_T), DIN_SEQ + "_length": i64[len_off:len_off + B]}
        target = {"feedid": i64[out_off[("target", "feedid")]:out_off[("target", "feedid")] + B]}
        return dense, category, sequence, target
