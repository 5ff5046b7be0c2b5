// Sorted nn.Embedding gradient (training, SURVEY.md §8(f) #2 "embedding-gradient scatter-add
// (sorted segment-reduce)"): grad[idx[i]] += dx[i, out_col : out_col + dim] for a long index list
// with hot rows — the behaviour sequences of DIN / BST, where every padded position maps to row 0
// (dcn.py:69, bst.py:142-150) and plain per-element atomics serialise on that row.
//
//   1. keys = idx (32-bit; out-of-range -> rows, flagged and skipped), values = positions 0..n-1
//   2. rocprim::radix_sort_pairs on the keys (only the bits the table needs)
//   3. workgroups take 64 consecutive sorted positions; per column a thread sums each run of equal
//      keys in order and adds it with one atomic per (distinct row in the chunk, column): a row hit
//      65k times costs 1k atomics per column instead of 65k.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"

namespace rk {

constexpr int kSortChunk = 64;

__global__ __launch_bounds__(256) void emb_sort_prep_kernel(const int64_t* __restrict__ idx, int64_t stride,
                                                            int64_t n, int64_t rows, uint32_t* __restrict__ keys,
                                                            uint32_t* __restrict__ pos, uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = idx[i * stride];
  const bool ok = r >= 0 && r < rows;
  if (!ok) flag_oob(flags);
  keys[i] = ok ? (uint32_t)r : (uint32_t)rows;
  pos[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void emb_sorted_reduce_kernel(const uint32_t* __restrict__ keys,
                                                                const uint32_t* __restrict__ pos, int64_t n,
                                                                const float* __restrict__ dx, int64_t ld_dx,
                                                                int out_col, int dim, uint32_t rows,
                                                                float* __restrict__ grad, int64_t ld_grad) {
  __shared__ uint32_t sk[kSortChunk], sp[kSortChunk];
  const int64_t i0 = (int64_t)blockIdx.x * kSortChunk;
  const int cnt = (int)min<int64_t>(kSortChunk, n - i0);
  if (threadIdx.x < cnt) {
    sk[threadIdx.x] = keys[i0 + threadIdx.x];
    sp[threadIdx.x] = pos[i0 + threadIdx.x];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < dim; c += blockDim.x) {
    float acc = 0.f;
    for (int j = 0; j < cnt; ++j) {
      acc += dx[(int64_t)sp[j] * ld_dx + out_col + c];
      if (j + 1 == cnt || sk[j + 1] != sk[j]) {
        if (sk[j] != rows && acc != 0.f) atomicAdd(grad + (int64_t)sk[j] * ld_grad + c, acc);
        acc = 0.f;
      }
    }
  }
}

// Behaviour-sequence form without the sort (B x T index matrix, dim even and <= 128): one wave per
// sample walks its T positions in order (lane = 2 columns), summing each run of equal consecutive
// ids and flushing one atomic per column per run.  A padded tail (the same id repeated to T, the
// hot row of the sorted path) is the sample's last run: the kSeqWaves samples of a workgroup merge
// equal tail ids in LDS first, so a padding row costs one atomic per column per 16 samples.
constexpr int kSeqWaves = 16;
__global__ __launch_bounds__(64 * kSeqWaves) void emb_seq_runs_kernel(const int64_t* __restrict__ idx, int64_t ld_idx, int64_t B,
                                                           int T, int64_t rows, const float* __restrict__ dx,
                                                           int64_t ld_dx, int out_col, int dim,
                                                           float* __restrict__ grad, int64_t ld_grad,
                                                           uint32_t* flags) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  __shared__ f32x2 tail[kSeqWaves][64];
  __shared__ int64_t tail_key[kSeqWaves];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * kSeqWaves + w;
  const int c = 2 * lane;
  const bool on = c < dim;
  int64_t key = -1;
  f32x2 acc = {0.f, 0.f};
  if (b < B) {
    const int64_t* ids = idx + b * ld_idx;
    const float* rowp = dx + b * T * ld_dx + out_col + c;
    key = ids[0];
    for (int t0 = 0; t0 < T; t0 += 8) {
      int64_t id[9];
      f32x2 v[8];
#pragma unroll
      for (int j = 0; j < 9; ++j) id[j] = t0 + j < T ? ids[t0 + j] : 0;  // past the end: never compared
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = (on && t0 + j < T) ? *reinterpret_cast<const f32x2*>(rowp + (int64_t)(t0 + j) * ld_dx)
                                  : f32x2{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (t0 + j >= T) break;
        acc += v[j];
        if (t0 + j + 1 < T && id[j + 1] != id[j]) {  // a run ends before the sample's last position
          const int64_t r = id[j];
          if (r >= 0 && r < rows) {
            if (on) {
              float* g = grad + r * ld_grad + c;
              if (acc[0] != 0.f) atomicAdd(g, acc[0]);
              if (acc[1] != 0.f) atomicAdd(g + 1, acc[1]);
            }
          } else if (lane == 0) {
            flag_oob(flags);
          }
          acc = f32x2{0.f, 0.f};
          key = id[j + 1];
        }
      }
    }
    if (!(key >= 0 && key < rows)) {
      if (lane == 0) flag_oob(flags);
      key = -1;
    }
  }
  tail[w][lane] = acc;
  if (lane == 0) tail_key[w] = key;
  __syncthreads();
  if (key < 0 || !on) return;
  for (int u = 0; u < w; ++u)
    if (tail_key[u] == key) return;  // merged by the first wave holding this tail id
  f32x2 sum = acc;
  for (int u = w + 1; u < kSeqWaves; ++u)
    if (tail_key[u] == key) sum += tail[u][lane];
  float* g = grad + key * ld_grad + c;
  if (sum[0] != 0.f) atomicAdd(g, sum[0]);
  if (sum[1] != 0.f) atomicAdd(g + 1, sum[1]);
}

struct SortPlan {
  size_t sort_bytes = 0, total = 0;
  size_t off_k0 = 0, off_k1 = 0, off_p0 = 0, off_p1 = 0, off_tmp = 0;
};

static size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

static SortPlan sort_plan(int64_t n) {
  SortPlan p;
  const unsigned un = (unsigned)n;
  (void)rocprim::radix_sort_pairs(nullptr, p.sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (uint32_t*)nullptr, un);
  const size_t a = align_up((size_t)n * sizeof(uint32_t));
  p.off_k0 = 0;
  p.off_k1 = a;
  p.off_p0 = 2 * a;
  p.off_p1 = 3 * a;
  p.off_tmp = 4 * a;
  p.total = p.off_tmp + align_up(p.sort_bytes);
  return p;
}

}  // namespace rk

using namespace rk;

RK_API int rk_embedding_backward_sorted_workspace_size(int64_t n, int64_t* bytes) {
  if (n < 0 || n >= (int64_t)UINT32_MAX || !bytes)
    return fail(RK_ERR_INVALID, "rk_embedding_backward_sorted_workspace_size: bad n");
  *bytes = (int64_t)sort_plan(n).total;
  return RK_OK;
}

RK_API int rk_embedding_backward_sorted(const rk_segment* grad, int64_t n, const float* dx, int64_t ld_dx,
                                        void* workspace, int64_t ws_bytes, void* stream) {
  if (!grad || !grad->src || !grad->idx || grad->dim <= 0 || grad->rows <= 0 || grad->rows >= (int64_t)UINT32_MAX ||
      grad->out_col < 0 || grad->out_col + grad->dim > ld_dx || !dx || n < 0 || n >= (int64_t)UINT32_MAX ||
      !workspace)
    return fail(RK_ERR_INVALID, "rk_embedding_backward_sorted: bad arguments");
  if (n == 0) return RK_OK;
  const SortPlan p = sort_plan(n);
  if (ws_bytes < (int64_t)p.total)
    return fail(RK_ERR_INVALID, "rk_embedding_backward_sorted: workspace %lld < %zu bytes", (long long)ws_bytes,
                p.total);
  char* ws = static_cast<char*>(workspace);
  uint32_t *k0 = (uint32_t*)(ws + p.off_k0), *k1 = (uint32_t*)(ws + p.off_k1);
  uint32_t *p0 = (uint32_t*)(ws + p.off_p0), *p1 = (uint32_t*)(ws + p.off_p1);
  hipStream_t st = (hipStream_t)stream;
  emb_sort_prep_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(grad->idx, grad->idx_stride, n, grad->rows, k0,
                                                                     p0, device_flags());
  int bits = 1;  // keys lie in [0, rows]
  while (bits < 32 && ((uint64_t)1 << bits) <= (uint64_t)grad->rows) ++bits;
  size_t tb = p.sort_bytes;
  if (rocprim::radix_sort_pairs(ws + p.off_tmp, tb, k0, k1, p0, p1, (unsigned)n, 0, bits, st) != hipSuccess)
    return fail(RK_ERR_LAUNCH, "rk_embedding_backward_sorted: radix sort failed");
  // (a wave-per-64-positions float2 variant measured 100 us vs 76 us here at BST configs[3]: the
  // padding row's per-column atomics, not the row loads, bound this kernel)
  emb_sorted_reduce_kernel<<<(unsigned)((n + kSortChunk - 1) / kSortChunk), 256, 0, st>>>(
      k1, p1, n, dx, ld_dx, grad->out_col, grad->dim, (uint32_t)grad->rows, const_cast<float*>(grad->src),
      grad->src_ld);
  return check_launch("rk_embedding_backward_sorted");
}

RK_API int rk_embedding_backward_seq(const rk_segment* grad, int64_t batch, int32_t T, const float* dx, int64_t ld_dx,
                                     void* stream) {
  if (!grad || !grad->src || !grad->idx || grad->dim <= 0 || grad->rows <= 0 || grad->out_col < 0 ||
      grad->out_col + grad->dim > ld_dx || !dx || batch < 0 || T <= 0 || grad->idx_stride < T)
    return fail(RK_ERR_INVALID, "rk_embedding_backward_seq: bad arguments");
  if (grad->dim % 2 || grad->dim > 128 || grad->out_col % 2 || ld_dx % 2 || grad->src_ld % 2 ||
      ((reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(grad->src)) & 7))
    return fail(RK_ERR_UNSUPPORTED, "rk_embedding_backward_seq: needs an even dim <= 128 and 8-B aligned rows");
  if (batch == 0) return RK_OK;
  emb_seq_runs_kernel<<<(unsigned)((batch + kSeqWaves - 1) / kSeqWaves), 64 * kSeqWaves, 0, (hipStream_t)stream>>>(
      grad->idx, grad->idx_stride, batch, T, grad->rows, dx, ld_dx, grad->out_col, grad->dim,
      const_cast<float*>(grad->src), grad->src_ld, device_flags());
  return check_launch("rk_embedding_backward_seq");
}
