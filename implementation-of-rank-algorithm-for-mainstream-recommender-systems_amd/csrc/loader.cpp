// Host input path: vocabulary bucketing (hazard H1) for raw ID string columns.  Contract and
// reference lines: include/rankops_io.h.  Plain C++17 host code (no GPU), built into
// librankops.so next to the kernels.
//
// A vocabulary is an open-addressing hash table (linear probing, power-of-two capacity >= 2x
// keys) over an arena of key bytes; lookups compare the 64-bit hash, then the length, then the
// bytes.  Columns arrive in the Apache Arrow layout so a pyarrow / parquet column is bucketed
// in place, split over up to 16 threads.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rankops.h"
#include "../../include/rankops_io.h"
#include "vocab_hash.h"

#define RK_API extern "C" __attribute__((visibility("default")))

namespace rk {
int fail(int code, const char* fmt, ...);  // runtime.hip: records rk_last_error()
}

namespace {

// Length of the str.isspace() character that starts at p (0 if none), UTF-8.
inline size_t space_at(const unsigned char* p, const unsigned char* end) {
  const unsigned c = p[0];
  if ((c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x20)) return 1;
  if (c == 0xC2 && end - p >= 2 && (p[1] == 0x85 || p[1] == 0xA0)) return 2;  // U+0085, U+00A0
  if (end - p >= 3) {
    if (c == 0xE1 && p[1] == 0x9A && p[2] == 0x80) return 3;  // U+1680
    if (c == 0xE2 && p[1] == 0x80 && (p[2] <= 0x8A || p[2] == 0xA8 || p[2] == 0xA9 || p[2] == 0xAF) && p[2] >= 0x80)
      return 3;                                                // U+2000-200A, U+2028, U+2029, U+202F
    if (c == 0xE2 && p[1] == 0x81 && p[2] == 0x9F) return 3;  // U+205F
    if (c == 0xE3 && p[1] == 0x80 && p[2] == 0x80) return 3;  // U+3000
  }
  return 0;
}

// Length of the str.isspace() character that ends at end (0 if none), UTF-8.
inline size_t space_before(const unsigned char* begin, const unsigned char* end) {
  if (end - begin >= 1 && space_at(end - 1, end) == 1) return 1;
  if (end - begin >= 2 && space_at(end - 2, end) == 2) return 2;
  if (end - begin >= 3 && space_at(end - 3, end) == 3) return 3;
  return 0;
}

inline bool bit_valid(const uint8_t* bits, int64_t off, int64_t i) {
  if (!bits) return true;
  const int64_t b = off + i;
  return (bits[b >> 3] >> (b & 7)) & 1;
}

inline void value_span(const void* offsets, int bits, int64_t i, int64_t& a, int64_t& b) {
  if (bits == 32) {
    const int32_t* o = static_cast<const int32_t*>(offsets);
    a = o[i];
    b = o[i + 1];
  } else {
    const int64_t* o = static_cast<const int64_t*>(offsets);
    a = o[i];
    b = o[i + 1];
  }
}

int thread_count(int requested, int64_t n) {
  int t = requested > 0 ? requested : (int)std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 16u);
  const int64_t per = 8192;  // below this many values per thread, spawning costs more than it saves
  t = (int)std::max<int64_t>(1, std::min<int64_t>(t, (n + per - 1) / per));
  return t;
}

template <class F>
void parallel_for(int64_t n, int threads, F&& body) {
  if (threads <= 1) {
    body(0, n);
    return;
  }
  std::vector<std::thread> pool;
  const int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t a = t * chunk, b = std::min(n, a + chunk);
    if (a >= b) break;
    pool.emplace_back([&body, a, b] { body(a, b); });
  }
  for (auto& th : pool) th.join();
}

}  // namespace

using rk::VocabSlot;

struct rk_vocab {
  std::vector<char> arena;
  std::vector<VocabSlot> slots;
  uint64_t mask = 0;
  int64_t size = 0;

  void reserve(size_t keys) {
    size_t cap = 16;
    while (cap < 2 * keys + 2) cap <<= 1;
    slots.assign(cap, VocabSlot{0, -1, 0, 0});
    mask = cap - 1;
  }
  void put(const char* k, size_t n, int64_t idx) {
    const uint64_t h = rk::vocab_hash(k, (uint32_t)n);
    for (uint64_t s = h & mask;; s = (s + 1) & mask) {
      VocabSlot& e = slots[s];
      if (e.idx < 0) {
        e.h = h;
        e.idx = idx;
        e.off = (uint32_t)arena.size();
        e.len = (uint32_t)n;
        arena.insert(arena.end(), k, k + n);
        return;
      }
      if (e.h == h && e.len == n && std::memcmp(arena.data() + e.off, k, n) == 0) {
        e.idx = idx;  // a later duplicate line overwrites, like the dict comprehension
        return;
      }
    }
  }
  // index of key k, or -1 when it is not in the vocabulary
  int64_t find(const char* k, size_t n) const {
    const uint64_t h = rk::vocab_hash(k, (uint32_t)n);
    for (uint64_t s = h & mask;; s = (s + 1) & mask) {
      const VocabSlot& e = slots[s];
      if (e.idx < 0) return -1;
      if (e.h == h && e.len == n && std::memcmp(arena.data() + e.off, k, n) == 0) return e.idx;
    }
  }
  int64_t get(const char* k, size_t n) const {
    const int64_t r = find(k, n);
    return r < 0 ? 0 : r;  // not in the vocabulary -> row 0 (H1)
  }
};

using namespace rk;

RK_API rk_vocab* rk_vocab_parse(const char* text, int64_t nbytes, int32_t skip_empty_lines) {
  if (nbytes < 0 || (!text && nbytes > 0)) {
    fail(RK_ERR_INVALID, "rk_vocab_parse: bad buffer");
    return nullptr;
  }
  if (nbytes >= (int64_t)UINT32_MAX) {
    fail(RK_ERR_UNSUPPORTED, "rk_vocab_parse: %lld bytes (max 4 GiB)", (long long)nbytes);
    return nullptr;
  }
  const unsigned char* p = reinterpret_cast<const unsigned char*>(text);
  const unsigned char* end = p + nbytes;
  // lines as Python's universal-newline file iteration yields them
  std::vector<std::pair<const unsigned char*, const unsigned char*>> lines;
  for (const unsigned char* s = p; s < end;) {
    const unsigned char* e = s;
    while (e < end && *e != '\n' && *e != '\r') ++e;
    lines.emplace_back(s, e);
    if (e < end && *e == '\r' && e + 1 < end && e[1] == '\n') ++e;
    s = e + 1;
  }
  rk_vocab* v = new rk_vocab();
  v->reserve(lines.size());
  v->arena.reserve((size_t)nbytes);
  int64_t idx = 0;
  for (auto [a, b] : lines) {  // str.strip()
    for (size_t k; a < b && (k = space_at(a, b)) != 0;) a += k;
    for (size_t k; b > a && (k = space_before(a, b)) != 0;) b -= k;
    if (skip_empty_lines && a == b) continue;
    v->put(reinterpret_cast<const char*>(a), (size_t)(b - a), idx++);
  }
  v->size = idx;
  return v;
}

RK_API rk_vocab* rk_vocab_load(const char* path, int32_t skip_empty_lines) {
  if (!path) {
    fail(RK_ERR_INVALID, "rk_vocab_load: null path");
    return nullptr;
  }
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    fail(RK_ERR_INVALID, "rk_vocab_load: cannot open %s", path);
    return nullptr;
  }
  std::vector<char> buf;
  char tmp[1 << 16];
  size_t got;
  while ((got = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
  const bool err = std::ferror(f);
  std::fclose(f);
  if (err) {
    fail(RK_ERR_RUNTIME, "rk_vocab_load: read error on %s", path);
    return nullptr;
  }
  return rk_vocab_parse(buf.data(), (int64_t)buf.size(), skip_empty_lines);
}

RK_API int64_t rk_vocab_size(const rk_vocab* v) { return v ? v->size : -1; }

RK_API void rk_vocab_free(rk_vocab* v) { delete v; }

RK_API int rk_vocab_export_size(const rk_vocab* v, int64_t* slot_bytes, int64_t* arena_bytes, uint64_t* mask) {
  if (!v || !slot_bytes || !arena_bytes || !mask) return fail(RK_ERR_INVALID, "rk_vocab_export_size: null argument");
  *slot_bytes = (int64_t)(v->slots.size() * sizeof(VocabSlot));
  *arena_bytes = (int64_t)std::max<size_t>(v->arena.size(), 1);
  *mask = v->mask;
  return RK_OK;
}

RK_API int rk_vocab_export(const rk_vocab* v, void* slots_out, void* arena_out) {
  if (!v || !slots_out || !arena_out) return fail(RK_ERR_INVALID, "rk_vocab_export: null argument");
  std::memcpy(slots_out, v->slots.data(), v->slots.size() * sizeof(VocabSlot));
  if (!v->arena.empty()) std::memcpy(arena_out, v->arena.data(), v->arena.size());
  return RK_OK;
}

static int check_column(const char* who, const rk_vocab* v, bool need_vocab, const char* data, const void* offsets,
                        int32_t offset_bits, int64_t n) {
  if (n < 0) return fail(RK_ERR_INVALID, "%s: n = %lld", who, (long long)n);
  if (need_vocab && !v) return fail(RK_ERR_INVALID, "%s: null vocabulary", who);
  if (offset_bits != 32 && offset_bits != 64) return fail(RK_ERR_INVALID, "%s: offset_bits %d", who, offset_bits);
  if (n > 0 && (!offsets || !data)) return fail(RK_ERR_INVALID, "%s: null column buffers", who);
  return RK_OK;
}

RK_API int rk_bucketize(const rk_vocab* v, const char* data, const void* offsets, int32_t offset_bits,
                        const uint8_t* valid_bits, int64_t valid_offset, int64_t n, int64_t* out, int64_t out_stride,
                        int32_t threads) {
  if (int rc = check_column("rk_bucketize", v, true, data, offsets, offset_bits, n)) return rc;
  if (n > 0 && (!out || out_stride < 1)) return fail(RK_ERR_INVALID, "rk_bucketize: bad output");
  parallel_for(n, thread_count(threads, n), [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      int64_t r = 0;
      if (bit_valid(valid_bits, valid_offset, i)) {
        int64_t s, e;
        value_span(offsets, offset_bits, i, s, e);
        r = v->get(data + s, (size_t)(e - s));
      }
      out[i * out_stride] = r;
    }
  });
  return RK_OK;
}

RK_API int rk_sequence_lengths(const char* data, const void* offsets, int32_t offset_bits, const uint8_t* valid_bits,
                               int64_t valid_offset, int64_t n, char sep, int64_t* lengths, int64_t* max_len,
                               int32_t threads) {
  if (int rc = check_column("rk_sequence_lengths", nullptr, false, data, offsets, offset_bits, n)) return rc;
  if (n > 0 && !lengths) return fail(RK_ERR_INVALID, "rk_sequence_lengths: null lengths");
  const int nt = thread_count(threads, n);
  std::vector<int64_t> part(nt, 0);
  const int64_t chunk = (n + nt - 1) / std::max(nt, 1);
  parallel_for(n, nt, [&](int64_t a, int64_t b) {
    int64_t m = 0;
    for (int64_t i = a; i < b; ++i) {
      int64_t len = 0;
      if (bit_valid(valid_bits, valid_offset, i)) {
        int64_t s, e;
        value_span(offsets, offset_bits, i, s, e);
        len = 1 + std::count(data + s, data + e, sep);  // "".split(',') == ['']
      }
      lengths[i] = len;
      m = std::max(m, len);
    }
    part[chunk ? a / chunk : 0] = m;
  });
  if (max_len) *max_len = n ? *std::max_element(part.begin(), part.end()) : 0;
  return RK_OK;
}

RK_API int rk_bucketize_sequences(const rk_vocab* v, const char* data, const void* offsets, int32_t offset_bits,
                                  const uint8_t* valid_bits, int64_t valid_offset, int64_t n, char sep, int64_t T,
                                  int64_t* out, int64_t ld_out, int64_t* lengths, int32_t threads) {
  if (int rc = check_column("rk_bucketize_sequences", v, true, data, offsets, offset_bits, n)) return rc;
  if (T < 0 || ld_out < T || (n > 0 && T > 0 && !out)) return fail(RK_ERR_INVALID, "rk_bucketize_sequences: bad output");
  // a history row is ~tens of lookups: split by rows, sized by the lookups they carry
  parallel_for(n, thread_count(threads, n * std::max<int64_t>(1, std::min<int64_t>(T, 32))), [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      int64_t* row = out + i * ld_out;
      int64_t j = 0;
      if (bit_valid(valid_bits, valid_offset, i)) {
        int64_t s, e;
        value_span(offsets, offset_bits, i, s, e);
        const char* p = data + s;
        const char* end = data + e;
        while (j < T) {
          const char* q = static_cast<const char*>(std::memchr(p, sep, (size_t)(end - p)));
          const char* item_end = q ? q : end;
          row[j++] = v->get(p, (size_t)(item_end - p));
          if (!q) break;
          p = q + 1;
        }
      }
      if (lengths) lengths[i] = j;
      for (; j < T; ++j) row[j] = 0;
    }
  });
  return RK_OK;
}

// ---------------------------------------------------------------------------------------------
// FwFM LabelEncoder bucketing (fwfm.py:48-67), over one whole dataset column.
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int64_t kNaN = -2, kOOV = -1;

// int(s) for the ASCII forms Python accepts: whitespace, sign, digits with single '_' between
bool parse_py_int(const unsigned char* a, const unsigned char* b, int64_t& out) {
  for (size_t k; a < b && (k = space_at(a, b)) != 0;) a += k;
  for (size_t k; b > a && (k = space_before(a, b)) != 0;) b -= k;
  bool neg = false;
  if (a < b && (*a == '+' || *a == '-')) neg = *a++ == '-';
  if (a == b || *a == '_' || b[-1] == '_') return false;
  unsigned __int128 v = 0;
  for (const unsigned char* p = a; p < b; ++p) {
    if (*p == '_') {
      if (p[1] == '_') return false;
      continue;
    }
    if (*p < '0' || *p > '9') return false;
    v = v * 10 + (*p - '0');
    if (v > (unsigned __int128)INT64_MAX + 1) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  out = neg ? (int64_t)(0 - (uint64_t)v) : (int64_t)v;
  return true;
}

}  // namespace

RK_API int rk_label_encode(const rk_vocab* v, const char* data, const void* offsets, int32_t offset_bits,
                           const uint8_t* valid_bits, int64_t valid_offset, int64_t n, int64_t* out,
                           int64_t* mode_index, int32_t threads) {
  if (int rc = check_column("rk_label_encode", nullptr, false, data, offsets, offset_bits, n)) return rc;
  if (n > 0 && !out) return fail(RK_ERR_INVALID, "rk_label_encode: null output");
  if (mode_index) *mode_index = -1;
  const int nt = thread_count(threads, n);
  auto value = [&](int64_t i, int64_t& s, int64_t& e) -> bool {  // false: NaN (null or the string "None")
    if (!bit_valid(valid_bits, valid_offset, i)) return false;
    value_span(offsets, offset_bits, i, s, e);
    return !(e - s == 4 && std::memcmp(data + s, "None", 4) == 0);
  };
  if (!v || v->size == 0) {
    // no vocabulary: data[feature].fillna(0).astype(int) (fwfm.py:66-67)
    std::vector<int64_t> bad(nt, -1);
    const int64_t chunk = (n + nt - 1) / std::max(nt, 1);
    parallel_for(n, nt, [&](int64_t a, int64_t b) {
      for (int64_t i = a; i < b; ++i) {
        int64_t s, e, r = 0;
        if (value(i, s, e) && !parse_py_int(reinterpret_cast<const unsigned char*>(data + s),
                                            reinterpret_cast<const unsigned char*>(data + e), r)) {
          bad[chunk ? a / chunk : 0] = i;
          return;
        }
        out[i] = r;
      }
    });
    for (int64_t i : bad)
      if (i >= 0) {
        int64_t s, e;
        value_span(offsets, offset_bits, i, s, e);
        return fail(RK_ERR_INVALID, "rk_label_encode: invalid literal for int() with base 10: '%.*s'",
                    (int)std::min<int64_t>(e - s, 200), data + s);
      }
    return RK_OK;
  }
  // pass 1: vocabulary index, kOOV or kNaN per row; per-index counts; OOV rows per thread
  std::vector<uint64_t> counts((size_t)v->size, 0);
  std::vector<std::vector<int64_t>> oov_rows(nt);
  const int64_t chunk = (n + nt - 1) / std::max(nt, 1);
  parallel_for(n, nt, [&](int64_t a, int64_t b) {
    auto& mine = oov_rows[chunk ? a / chunk : 0];
    for (int64_t i = a; i < b; ++i) {
      int64_t s, e, r = kNaN;
      if (value(i, s, e)) {
        r = v->find(data + s, (size_t)(e - s));
        if (r >= 0)
          __atomic_fetch_add(&counts[(size_t)r], 1, __ATOMIC_RELAXED);
        else
          mine.push_back(i);
      }
      out[i] = r;
    }
  });
  // series.mode(dropna=True).values[0]: the most frequent value, ties -> the smallest string
  // (code-point order == UTF-8 byte order)
  std::vector<std::string_view> key_of((size_t)v->size);
  for (const VocabSlot& e : v->slots)
    if (e.idx >= 0) key_of[(size_t)e.idx] = std::string_view(v->arena.data() + e.off, e.len);
  uint64_t best = 0;
  std::string_view best_key;
  bool best_in_vocab = false;
  int64_t best_idx = -1;
  auto offer = [&](uint64_t c, std::string_view k, bool in_vocab, int64_t idx) {
    if (c == 0) return;
    if (c > best || (c == best && k < best_key)) {
      best = c;
      best_key = k;
      best_in_vocab = in_vocab;
      best_idx = idx;
    }
  };
  for (size_t r = 0; r < counts.size(); ++r) offer(counts[r], key_of[r], true, (int64_t)r);
  std::unordered_map<std::string_view, uint64_t> oov;
  for (auto& rows : oov_rows)
    for (int64_t i : rows) {
      int64_t s, e;
      value_span(offsets, offset_bits, i, s, e);
      ++oov[std::string_view(data + s, (size_t)(e - s))];
    }
  for (auto& [k, c] : oov) offer(c, k, false, -1);
  if (n == 0) return RK_OK;
  if (best == 0) {  // every value NaN: the mode is 'unknown'
    best_key = "unknown";
    best_idx = v->find("unknown", 7);
    best_in_vocab = best_idx >= 0;
  }
  if (!best_in_vocab)  // the reference's LabelEncoder.transform raises here
    return fail(RK_ERR_INVALID, "rk_label_encode: y contains previously unseen labels: '%.*s' (the column's mode)",
                (int)std::min<size_t>(best_key.size(), 200), best_key.data());
  // pass 2: NaN and out-of-vocabulary rows take the mode's index
  parallel_for(n, nt, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i)
      if (out[i] < 0) out[i] = best_idx;
  });
  if (mode_index) *mode_index = best_idx;
  return RK_OK;
}
