/*
 * rankops_io.h — host-side C ABI of the rankops input path: raw ID strings
 * -> int64 embedding rows with the reference's bucketing semantics (hazard H1), batch-assembled
 * for one host-to-device copy.  The rk_vocab_* / rk_bucketize* / rk_sequence_lengths calls are
 * host code (thread-safe for concurrent calls on one vocabulary); the *_device variants enqueue
 * the same lookup on a HIP stream against a vocabulary table exported to device memory
 * (rk_vocab_export), with all column buffers in device memory.
 *
 * Reference interfaces replaced (file:line in the reference snapshot):
 *   rk_vocab_load / rk_vocab_parse   _load_vocabulary + the vocab_indices dict comprehension:
 *                                    dcn.py:59-69,84-89; din.py:92-102,121-126;
 *                                    bst.py:29-33,100-110; deepfm.py:31-40,46-51;
 *                                    deepcrossing.py:51-61,76-81; with skip_empty_lines = 1
 *                                    afm.py:31-36 (and the table sizes of afm.py:147-150)
 *   rk_bucketize                     the per-row category / target lookups of __getitem__:
 *                                    dcn.py:94-104; din.py:131-143,158-163; bst.py:130-140;
 *                                    deepfm.py:56-66; afm.py:46-54; deepcrossing.py:86-100
 *   rk_label_encode                  FwFM's dataset-level LabelEncoder bucketing: fwfm.py:29-31
 *                                    ('None' -> NaN), fwfm.py:48-67 (mode fill, OOV -> mode,
 *                                    LabelEncoder.transform with classes_ = the vocabulary lines)
 *   rk_sequence_lengths,             DIN history: str.split(',') + per-item feedid lookup
 *   rk_bucketize_sequences           (din.py:145-157) and din_collate_fn's zero padding to the
 *                                    batch maximum (din.py:175-213); BST's one-item sequence
 *                                    zero-padded to max_seq_length (bst.py:142-150)
 *
 * Semantics (bit-exact with the Python code above):
 *   - vocabulary file = text lines split like Python's universal-newline iteration ("\n", "\r\n"
 *     and a lone "\r" end a line; a final line without terminator counts), each stripped like
 *     str.strip() (ASCII whitespace 0x09-0x0D, 0x1C-0x20 and the Unicode White_Space code points
 *     in UTF-8: U+0085, U+00A0, U+1680, U+2000-U+200A, U+2028, U+2029, U+202F, U+205F, U+3000);
 *     with skip_empty_lines, lines that strip to "" are dropped before numbering (afm.py);
 *   - index of a key = position of its LAST occurrence (dict comprehension overwrite);
 *     rk_vocab_size = number of lines kept (len(vocab)); tables have size + 1 rows (H1);
 *   - a value that is not in the vocabulary, or is null, maps to 0 (collides with entry 0);
 *     values are looked up exactly as given (no strip);
 *   - sequences: value.split(sep) (an empty string is one empty item), every item looked up;
 *     length = number of items; a null value is an empty sequence (row.get(col, []));
 *     rows are zero-padded (or truncated, lengths capped: bst.py:146) to T columns.
 *
 * String columns use the Apache Arrow layout: value i is data[offsets[i] .. offsets[i+1]),
 * offsets int32 (offset_bits = 32, Arrow "string") or int64 (64, "large_string"); validity is
 * an Arrow bitmap (bit (valid_offset + i), LSB first) or NULL for all valid.
 * threads <= 0 picks the hardware concurrency (capped at 16).
 */
#ifndef RANKOPS_IO_H
#define RANKOPS_IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rk_vocab rk_vocab;

/* Loads a vocabulary file; NULL on error (rk_last_error()). */
rk_vocab* rk_vocab_load(const char* path, int32_t skip_empty_lines);
/* Same parse from an in-memory file image of nbytes bytes. */
rk_vocab* rk_vocab_parse(const char* text, int64_t nbytes, int32_t skip_empty_lines);
int64_t rk_vocab_size(const rk_vocab* v);
void rk_vocab_free(rk_vocab* v);

/* out[i * out_stride] = index of value i, or 0. */
int rk_bucketize(const rk_vocab* v, const char* data, const void* offsets, int32_t offset_bits,
                 const uint8_t* valid_bits, int64_t valid_offset, int64_t n, int64_t* out,
                 int64_t out_stride, int32_t threads);

/* lengths[i] = number of sep-separated items of value i (0 for null); *max_len = max_i. */
int rk_sequence_lengths(const char* data, const void* offsets, int32_t offset_bits,
                        const uint8_t* valid_bits, int64_t valid_offset, int64_t n, char sep,
                        int64_t* lengths, int64_t* max_len, int32_t threads);

/* out[i, 0:T] = indices of the first min(len_i, T) items of value i, zero-filled after;
 * lengths[i] = min(len_i, T) (may be NULL).  out has row stride ld_out (>= T).              */
int rk_bucketize_sequences(const rk_vocab* v, const char* data, const void* offsets,
                           int32_t offset_bits, const uint8_t* valid_bits, int64_t valid_offset,
                           int64_t n, char sep, int64_t T, int64_t* out, int64_t ld_out,
                           int64_t* lengths, int32_t threads);

/* Device copy of a vocabulary: the hash table image (slot_bytes, 24-B slots) and key arena
 * (arena_bytes) to copy into device memory as they are; `mask` is passed to the *_device calls. */
/* FwFM LabelEncoder bucketing of one whole column (fwfm.py:48-67): a null or the string "None" is
 * NaN; out[i] = vocabulary index (last occurrence, no +1) of value i, with NaN and out-of-vocabulary
 * values replaced by the column's mode — the most frequent non-NaN value (ties: smallest string in
 * code-point order), "unknown" when every value is NaN — reported in *mode_index (may be NULL).
 * Fails with RK_ERR_INVALID ("y contains previously unseen labels") when the mode is not in the
 * vocabulary, where sklearn's LabelEncoder.transform raises.  v == NULL or an empty vocabulary:
 * the values are parsed as Python int() (ASCII digits, optional sign / '_' / whitespace), NaN -> 0
 * (fwfm.py:66-67).  Load the vocabulary with skip_empty_lines = 0 (fwfm.py:43-44).             */
int rk_label_encode(const rk_vocab* v, const char* data, const void* offsets, int32_t offset_bits,
                    const uint8_t* valid_bits, int64_t valid_offset, int64_t n, int64_t* out,
                    int64_t* mode_index, int32_t threads);
int rk_vocab_export_size(const rk_vocab* v, int64_t* slot_bytes, int64_t* arena_bytes, uint64_t* mask);
int rk_vocab_export(const rk_vocab* v, void* slots_out, void* arena_out);

/* rk_bucketize / rk_bucketize_sequences on the GPU: slots/arena = device copies of the export,
 * data/offsets/valid_bits/out/lengths device pointers; enqueued on `stream`, no sync.        */
int rk_bucketize_device(const void* slots, uint64_t mask, const char* arena, const char* data,
                        const void* offsets, int32_t offset_bits, const uint8_t* valid_bits,
                        int64_t valid_offset, int64_t n, int64_t* out, int64_t out_stride,
                        void* stream);
int rk_bucketize_sequences_device(const void* slots, uint64_t mask, const char* arena,
                                  const char* data, const void* offsets, int32_t offset_bits,
                                  const uint8_t* valid_bits, int64_t valid_offset, int64_t n,
                                  char sep, int64_t T, int64_t* out, int64_t ld_out,
                                  int64_t* lengths, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RANKOPS_IO_H */
