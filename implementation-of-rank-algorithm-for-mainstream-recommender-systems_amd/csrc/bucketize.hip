// Device bucketing (hazard H1) of raw ID string columns against a vocabulary hash table exported
// from the host loader (rk_vocab_export) and copied to HBM.  Same hash, same slot image and the
// same semantics as rk_bucketize / rk_bucketize_sequences (include/rankops_io.h), so a batch's
// raw Arrow string buffers go to the GPU in the batch's one host-to-device copy and the int64
// rows are produced next to the embedding tables instead of by host threads.
//
// rk_bucketize_device: one lane per value.  rk_bucketize_sequences_device: one wave per row — the
// lanes scan the row's bytes 64 at a time, locate the separators with a ballot, record item
// starts in LDS, then look the items up in parallel (lane j: items j, j+64, ...).
#include "common.h"
#include "vocab_hash.h"

namespace rk {

namespace {

struct StrCol {
  const char* data;
  const void* offsets;
  int bits;
  const uint8_t* valid;
  int64_t valid_off;
};

__device__ __forceinline__ bool col_valid(const StrCol& c, int64_t i) {
  if (!c.valid) return true;
  const int64_t b = c.valid_off + i;
  return (c.valid[b >> 3] >> (b & 7)) & 1;
}

__device__ __forceinline__ void col_span(const StrCol& c, int64_t i, int64_t& a, int64_t& b) {
  if (c.bits == 32) {
    const int32_t* o = static_cast<const int32_t*>(c.offsets);
    a = o[i];
    b = o[i + 1];
  } else {
    const int64_t* o = static_cast<const int64_t*>(c.offsets);
    a = o[i];
    b = o[i + 1];
  }
}

__global__ __launch_bounds__(256) void bucketize_kernel(const VocabSlot* __restrict__ slots, uint64_t mask,
                                                        const char* __restrict__ arena, StrCol col, int64_t n,
                                                        int64_t* __restrict__ out, int64_t stride) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = 0;
    if (col_valid(col, i)) {
      int64_t a, b;
      col_span(col, i, a, b);
      r = vocab_find(slots, mask, arena, col.data + a, (uint32_t)(b - a));
    }
    out[i * stride] = r;
  }
}

constexpr int kSeqWaves = 4;      // rows per 256-thread block (one wave per row)
constexpr int kMaxItemsLds = 512;  // item starts held in LDS per scan pass

// LDS hand-off between lanes of ONE wave: the wave's LDS writes are complete (and the compiler
// may not move LDS accesses across) — no block barrier, the waves work on different rows.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__global__ __launch_bounds__(256) void bucketize_sequences_kernel(const VocabSlot* __restrict__ slots, uint64_t mask,
                                                                  const char* __restrict__ arena, StrCol col,
                                                                  int64_t n, char sep, int64_t T,
                                                                  int64_t* __restrict__ out, int64_t ld_out,
                                                                  int64_t* __restrict__ lengths) {
  __shared__ int64_t starts_lds[kSeqWaves][kMaxItemsLds + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t* starts = starts_lds[w];
  for (int64_t row = blockIdx.x * (int64_t)kSeqWaves + w; row < n; row += (int64_t)gridDim.x * kSeqWaves) {
    int64_t* orow = out + row * ld_out;
    int64_t count = 0;  // items written (<= T); all control flow below is wave-uniform
    if (col_valid(col, row)) {
      int64_t a, b;
      col_span(col, row, a, b);
      int64_t cur = a;  // start of the first item not written yet
      while (true) {
        // pass: starts[0] = cur, then the start (separator + 1) of every following item, scanning
        // 64 bytes per step, until the row ends, LDS is full or enough items for T are known
        if (lane == 0) starts[0] = cur;
        int nst = 1;
        bool row_end = false;
        for (int64_t scan = cur;;) {
          const int64_t p = scan + lane;
          const bool is_sep = p < b && col.data[p] == sep;
          const uint64_t m = __ballot(is_sep);
          const int before = __popcll(m & ((1ull << lane) - 1));
          const int room = kMaxItemsLds + 1 - nst;
          if (is_sep && before < room) starts[nst + before] = p + 1;
          const int found = __popcll(m);
          if (found > room) {  // LDS full: the last recorded item is resumed in the next pass
            nst += room;
            break;
          }
          nst += found;
          scan += 64;
          if (scan >= b) {
            row_end = true;
            break;
          }
          if (count + nst - 1 >= T) break;  // enough complete items
        }
        wave_lds_sync();
        // items k < nst - 1 end at the next separator; the last one ends at b only if the row ended
        const int complete = row_end ? nst : nst - 1;
        const int take = (int)std::min<int64_t>(complete, T - count);
        for (int k = lane; k < take; k += 64) {
          const int64_t s = starts[k];
          const int64_t e = k + 1 < nst ? starts[k + 1] - 1 : b;
          orow[count + k] = vocab_find(slots, mask, arena, col.data + s, (uint32_t)(e - s));
        }
        count += take;
        if (row_end || count >= T) break;
        cur = starts[nst - 1];
        wave_lds_sync();  // every lane has read starts[] before the next pass overwrites it
      }
    }
    for (int64_t j = count + lane; j < T; j += 64) orow[j] = 0;
    if (lengths && lane == 0) lengths[row] = count;
  }
}

}  // namespace

}  // namespace rk

using namespace rk;

static int check_dev_args(const char* who, const void* slots, const char* arena, const char* data, const void* offsets,
                          int32_t bits, int64_t n) {
  if (n < 0) return fail(RK_ERR_INVALID, "%s: n = %lld", who, (long long)n);
  if (bits != 32 && bits != 64) return fail(RK_ERR_INVALID, "%s: offset_bits %d", who, bits);
  if (!slots || !arena) return fail(RK_ERR_INVALID, "%s: null vocabulary table", who);
  if (n > 0 && (!data || !offsets)) return fail(RK_ERR_INVALID, "%s: null column buffers", who);
  return RK_OK;
}

RK_API int rk_bucketize_device(const void* slots, uint64_t mask, const char* arena, const char* data,
                               const void* offsets, int32_t offset_bits, const uint8_t* valid_bits,
                               int64_t valid_offset, int64_t n, int64_t* out, int64_t out_stride, void* stream) {
  if (int rc = check_dev_args("rk_bucketize_device", slots, arena, data, offsets, offset_bits, n)) return rc;
  if (n == 0) return RK_OK;
  if (!out || out_stride < 1) return fail(RK_ERR_INVALID, "rk_bucketize_device: bad output");
  StrCol c{data, offsets, offset_bits, valid_bits, valid_offset};
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8 * num_cus());
  bucketize_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(static_cast<const VocabSlot*>(slots), mask,
                                                                      arena, c, n, out, out_stride);
  return check_launch("rk_bucketize_device");
}

RK_API int rk_bucketize_sequences_device(const void* slots, uint64_t mask, const char* arena, const char* data,
                                         const void* offsets, int32_t offset_bits, const uint8_t* valid_bits,
                                         int64_t valid_offset, int64_t n, char sep, int64_t T, int64_t* out,
                                         int64_t ld_out, int64_t* lengths, void* stream) {
  if (int rc = check_dev_args("rk_bucketize_sequences_device", slots, arena, data, offsets, offset_bits, n)) return rc;
  if (T < 0 || ld_out < T || (n > 0 && T > 0 && !out))
    return fail(RK_ERR_INVALID, "rk_bucketize_sequences_device: bad output");
  if (n == 0) return RK_OK;
  StrCol c{data, offsets, offset_bits, valid_bits, valid_offset};
  const int64_t blocks = std::min<int64_t>((n + kSeqWaves - 1) / kSeqWaves, 16 * num_cus());
  bucketize_sequences_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(
      static_cast<const VocabSlot*>(slots), mask, arena, c, n, sep, T, out, ld_out, lengths);
  return check_launch("rk_bucketize_sequences_device");
}
