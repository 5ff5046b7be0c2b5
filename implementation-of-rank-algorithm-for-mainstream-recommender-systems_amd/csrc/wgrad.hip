// Weight-gradient GEMM of the training backward: dW[n][k] = sum_r dZ[r][n] X[r][k]
// and the bias gradient db[n] = sum_r dZ[r][n] over a long reduction (r = batch rows, 131,072 for
// BST's per-position projections), the `loss.backward()` of every nn.Linear in the reference's
// train() loops (bst.py:59-64,73-75,86-90; dcn.py:147-150; din.py:272-285).
//
// Shape: output N x K <= 128 x 128 per tile, reduction R >> N, K.  rk_gemm's 64 x 64 split-K tiles
// read every operand column block twice (once per output tile sharing it) and combine with float
// atomics; here one 512-thread workgroup owns a whole 128 x 128 output tile for a slab of rows, so
// dZ and X are each read once from HBM, and the slabs' partial tiles go to a workspace summed in a
// fixed order by a second kernel (deterministic).
//   * 64-row steps staged into a k-major (transposed) LDS image [128 cols][64 rows + 4] per operand:
//     float4 global loads, a 4 x 4 register transpose, ds_write_b128; the next step's loads are in
//     flight during this step's MFMAs;
//   * wave w owns n rows 32 (w & 3) .. +32 and k columns 64 (w >> 2) .. +64: two
//     v_mfma_f32_32x32x2_f32 tiles; each lane reads 4 consecutive reduction rows of its column with
//     one ds_read_b128 (3 reads per 8 MFMAs; the row-major image needed 8, and measured 51 us);
//   * the bias sums come from the staged registers (each thread's four columns, all its rows) and
//     are folded across the workgroup once at the end.
#include "common.h"

namespace rk {

constexpr int kWgT = 128;        // output tile edge (n and k)
constexpr int kWgR = 64;         // rows per step
constexpr int kWgP = kWgR + 4;   // LDS pitch of the k-major image S[col][row] (floats)
constexpr int kWgThreads = 512;
static_assert(kWgR * kWgT == 16 * kWgThreads, "one 4 x 4 staging block per thread and operand");

// Staging: thread t owns the 4 x 4 block (rows 4 (t >> 5) .. +3 of the step, columns 4 (t & 31) .. +3)
// of each operand: four float4 row loads (a wave covers two rows x 512 B per instruction), then a
// register transpose and four ds_write_b128 into the k-major LDS image S[col][row] (pitch kWgP), so
// the MFMA loop reads 4 consecutive reduction rows per lane with one ds_read_b128.
// Raw loads only (out-of-range rows / columns read a clamped in-range address): the zeroing and
// masking happen in wg_store, so nothing consumes the loaded registers until the next step's store
// and the loads stay in flight across this step's MFMAs.
template <bool MASK>
__device__ __forceinline__ void wg_load(const float* __restrict__ P, int64_t ld, const float* __restrict__ mask,
                                        int64_t r0, int64_t re, int c0, int cols, int tid, f32x4 (&v)[4],
                                        f32x4 (&m)[4]) {
  const int c = 4 * (tid & 31);
  const int cc = c0 + c < cols ? c0 + c : c0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t r = min<int64_t>(r0 + 4 * (tid >> 5) + i, re - 1);
    v[i] = *reinterpret_cast<const f32x4*>(P + r * ld + cc);
    if (MASK) m[i] = *reinterpret_cast<const f32x4*>(mask + r * ld + cc);
  }
}

// Store a staged step (rows >= re / columns >= cols zeroed, mask applied) transposed into the
// k-major LDS image; adds the stored values to bsum (per column) when SUMS.
template <bool MASK, bool SUMS>
__device__ __forceinline__ void wg_store(float* __restrict__ S, int tid, const f32x4 (&v)[4], const f32x4 (&m)[4],
                                         int64_t r0, int64_t re, int c0, int cols, f32x4& bsum) {
  const bool cok = c0 + 4 * (tid & 31) < cols;
  f32x4 x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ok = cok && r0 + 4 * (tid >> 5) + i < re;
#pragma unroll
    for (int e = 0; e < 4; ++e) x[i][e] = (ok && (!MASK || m[i][e] > 0.f)) ? v[i][e] : 0.f;
    if (SUMS) bsum += x[i];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e)
    *reinterpret_cast<f32x4*>(S + (4 * (tid & 31) + e) * kWgP + 4 * (tid >> 5)) =
        f32x4{x[0][e], x[1][e], x[2][e], x[3][e]};
}

// grid (splits, n tiles, k tiles); partial tile of split s -> ws[s][n][k] (N x K), bias partial ->
// wsb[s][n].
template <bool MASK>
__global__ __launch_bounds__(kWgThreads) void wgrad_kernel(int64_t N, int64_t K, int64_t R, int64_t rps,
                                                           const float* __restrict__ A, int64_t lda,
                                                           const float* __restrict__ A_mask,
                                                           const float* __restrict__ B, int64_t ldb,
                                                           float* __restrict__ ws, float* __restrict__ wsb) {
  __shared__ float As2[2][kWgT * kWgP];  // double-buffered k-major images (139 KB, one workgroup per CU)
  __shared__ float Bs2[2][kWgT * kWgP];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 3, wk = w >> 2;
#ifdef RK_WGRAD_STAMP  // diagnostic build only (tools/wgrad_clock.cpp): per-workgroup clock stamps
  uint64_t t0 = 0, r0s = 0;
  if (tid == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0s = __builtin_amdgcn_s_memrealtime();
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
#endif
  const int n0 = blockIdx.y * kWgT, k0 = blockIdx.z * kWgT;
  const int64_t rb = (int64_t)blockIdx.x * rps;
  const int64_t re = min<int64_t>(R, rb + rps);
  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
  f32x4 bsum = {0.f, 0.f, 0.f, 0.f};
  const bool sums = wsb && blockIdx.z == 0;
  f32x4 va[4], vb[4], ma[4], mb[4];
  // lane half h = lane >> 5 takes reduction rows 8g + 4h + e at MFMA e of row group g (the same rows
  // for the A and B operands, so the k-permutation cancels in the sum)
  const int a_off = (32 * wm + (lane & 31)) * kWgP + 4 * (lane >> 5);
  const int b_off = (64 * wk + (lane & 31)) * kWgP + 4 * (lane >> 5);
  // prologue: step 0 into buffer 0, step 1's loads in flight
  wg_load<MASK>(A, lda, A_mask, rb, re, n0, (int)N, tid, va, ma);
  wg_load<false>(B, ldb, nullptr, rb, re, k0, (int)K, tid, vb, mb);
  if (sums)
    wg_store<MASK, true>(As2[0], tid, va, ma, rb, re, n0, (int)N, bsum);
  else
    wg_store<MASK, false>(As2[0], tid, va, ma, rb, re, n0, (int)N, bsum);
  wg_store<false, false>(Bs2[0], tid, vb, mb, rb, re, k0, (int)K, bsum);
  if (rb + kWgR < re) {
    wg_load<MASK>(A, lda, A_mask, rb + kWgR, re, n0, (int)N, tid, va, ma);
    wg_load<false>(B, ldb, nullptr, rb + kWgR, re, k0, (int)K, tid, vb, mb);
  }
  __syncthreads();
  int cb = 0;
  // one barrier per step: step s computes from buffer s & 1 while step s + 1's rows (loaded during
  // step s - 1) are written into the other buffer between the MFMA groups
  for (int64_t r0 = rb; r0 < re; r0 += kWgR, cb ^= 1) {
    const float* a_col = As2[cb] + a_off;
    const float* b_col = Bs2[cb] + b_off;
    const bool more = r0 + kWgR < re;
    f32x4 a[2], b0[2], b1[2];
    a[0] = *reinterpret_cast<const f32x4*>(a_col);
    b0[0] = *reinterpret_cast<const f32x4*>(b_col);
    b1[0] = *reinterpret_cast<const f32x4*>(b_col + 32 * kWgP);
#pragma unroll
    for (int g = 0; g < kWgR / 8; ++g) {
      const int cur = g & 1, nxt = cur ^ 1;
      if (g + 1 < kWgR / 8) {
        a[nxt] = *reinterpret_cast<const f32x4*>(a_col + 8 * (g + 1));
        b0[nxt] = *reinterpret_cast<const f32x4*>(b_col + 8 * (g + 1));
        b1[nxt] = *reinterpret_cast<const f32x4*>(b_col + 32 * kWgP + 8 * (g + 1));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc0 = mfma32(a[cur][e], b0[cur][e], acc0);
        acc1 = mfma32(a[cur][e], b1[cur][e], acc1);
      }
      if (g == 1 && more) {  // the next step's rows have had a whole step to arrive
        if (sums)
          wg_store<MASK, true>(As2[cb ^ 1], tid, va, ma, r0 + kWgR, re, n0, (int)N, bsum);
        else
          wg_store<MASK, false>(As2[cb ^ 1], tid, va, ma, r0 + kWgR, re, n0, (int)N, bsum);
        wg_store<false, false>(Bs2[cb ^ 1], tid, vb, mb, r0 + kWgR, re, k0, (int)K, bsum);
        if (r0 + 2 * kWgR < re) {
          wg_load<MASK>(A, lda, A_mask, r0 + 2 * kWgR, re, n0, (int)N, tid, va, ma);
          wg_load<false>(B, ldb, nullptr, r0 + 2 * kWgR, re, k0, (int)K, tid, vb, mb);
        }
      }
    }
    __syncthreads();
  }
  // partial tile: lane holds C[n0 + 32 wm + acc_row(r)][k0 + 64 wk + (lane & 31) (+32)]
  float* out = ws + (int64_t)blockIdx.x * N * K;
  const int64_t k = k0 + 64 * wk + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t n = n0 + 32 * wm + acc_row(r, lane);
    if (n < N) {
      if (k < K) out[n * K + k] = acc0[r];
      if (k + 32 < K) out[n * K + k + 32] = acc1[r];
    }
  }
#ifdef RK_WGRAD_STAMP
  if (tid == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    extern __device__ uint64_t g_wgrad_stamp[];
    uint64_t* st = g_wgrad_stamp + 4 * (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
    st[0] = t0; st[1] = t1; st[2] = r0s; st[3] = r1;
  }
#endif
  if (sums) {  // fold the 16 row groups holding the same four columns (threads t, t + 32, ...)
    __syncthreads();
    float* red = As2[0];  // [16][128]
    *reinterpret_cast<f32x4*>(red + (tid >> 5) * kWgT + 4 * (tid & 31)) = bsum;
    __syncthreads();
    if (tid < kWgT && n0 + tid < N) {
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) s += red[g * kWgT + tid];
      wsb[(int64_t)blockIdx.x * N + n0 + tid] = s;
    }
  }
}

// C[n][k] (+)= sum_s ws[s][n][k] (float4 per lane, the 16 waves of a workgroup split s, fixed-order
// LDS combine); the workgroups past the tile's float4 count do the same for row_sums from wsb.
__global__ __launch_bounds__(1024) void wgrad_reduce_kernel(const float* __restrict__ ws, const float* __restrict__ wsb,
                                                            int64_t S, int64_t N, int64_t K, float* __restrict__ C,
                                                            int64_t ldc, float* __restrict__ row_sums, int accumulate,
                                                            int64_t c_blocks) {
  __shared__ f32x4 red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool bias = blockIdx.x >= c_blocks;
  const int64_t count4 = bias ? N / 4 : N * K / 4;
  const int64_t e = (bias ? blockIdx.x - c_blocks : blockIdx.x) * 64 + lane;  // float4 index
  const float* src = bias ? wsb : ws;
  const int64_t stride = bias ? N : N * K;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (e < count4) {
#pragma unroll 4
    for (int64_t sp = w; sp < S; sp += 16) s += *reinterpret_cast<const f32x4*>(src + sp * stride + 4 * e);
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && e < count4) {
    f32x4 t = red[0][lane];
#pragma unroll
    for (int i = 1; i < 16; ++i) t += red[i][lane];
    if (bias) {
      float* d = row_sums + 4 * e;
#pragma unroll
      for (int c = 0; c < 4; ++c) d[c] = accumulate ? d[c] + t[c] : t[c];
    } else {
      const int64_t n = (4 * e) / K, k = (4 * e) % K;  // K % 4 == 0: the 4 values share a row
      float* d = C + n * ldc + k;
#pragma unroll
      for (int c = 0; c < 4; ++c) d[c] = accumulate ? d[c] + t[c] : t[c];
    }
  }
}

static int64_t wgrad_splits(int64_t N, int64_t K, int64_t R) {
  const int64_t tiles = ((N + kWgT - 1) / kWgT) * ((K + kWgT - 1) / kWgT);
  // one workgroup per CU and output tile.  Two per CU (4 waves / SIMD) measured no faster
  // (tools/wgrad_clock.cpp: 40.7 us for half the rows vs 42.9 us), and the partial tiles double.
  const int64_t want = std::max<int64_t>(1, num_cus() / tiles);
  const int64_t steps = (R + kWgR - 1) / kWgR;
  return std::max<int64_t>(1, std::min<int64_t>(want, steps));
}

}  // namespace rk

using namespace rk;

RK_API int64_t rk_gemm_wgrad_workspace_floats(int64_t N, int64_t K, int64_t R) {
  if (N <= 0 || K <= 0 || R < 0) return 0;
  return wgrad_splits(N, K, R) * (N * K + N);
}

RK_API int rk_gemm_wgrad(int64_t N, int64_t K, int64_t R, const float* A, int64_t lda, const float* A_mask,
                         const float* B, int64_t ldb, float* C, int64_t ldc, float* row_sums, int32_t accumulate,
                         float* workspace, int64_t workspace_floats, void* stream) {
  if (N <= 0 || K <= 0 || R < 0 || !C || ldc < K || (R > 0 && (!A || !B)) || lda < N || ldb < K)
    return fail(RK_ERR_INVALID, "rk_gemm_wgrad: bad shape / operand");
  const uintptr_t align = reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B) |
                          reinterpret_cast<uintptr_t>(A_mask) | reinterpret_cast<uintptr_t>(C) |
                          reinterpret_cast<uintptr_t>(row_sums) | reinterpret_cast<uintptr_t>(workspace);
  if ((N | K | lda | ldb | ldc) % 4 || (align & 15))
    return fail(RK_ERR_UNSUPPORTED, "rk_gemm_wgrad: needs N, K, lda, ldb, ldc multiples of 4 and 16-B aligned "
                                    "pointers (use rk_gemm)");
  if (!workspace || workspace_floats < rk_gemm_wgrad_workspace_floats(N, K, R))
    return fail(RK_ERR_INVALID, "rk_gemm_wgrad: workspace of %lld floats, needs %lld", (long long)workspace_floats,
                (long long)rk_gemm_wgrad_workspace_floats(N, K, R));
  hipStream_t st = (hipStream_t)stream;
  const int64_t S = wgrad_splits(N, K, R);
  int64_t rps = (R + S - 1) / S;
  rps = std::max<int64_t>(kWgR, (rps + kWgR - 1) / kWgR * kWgR);
  const int64_t splits = std::max<int64_t>(1, (R + rps - 1) / rps);
  float* wsb = workspace + splits * N * K;
  if (R > 0) {
    const dim3 grid((unsigned)splits, (unsigned)((N + kWgT - 1) / kWgT), (unsigned)((K + kWgT - 1) / kWgT));
    if (A_mask)
      wgrad_kernel<true><<<grid, kWgThreads, 0, st>>>(N, K, R, rps, A, lda, A_mask, B, ldb, workspace,
                                                      row_sums ? wsb : nullptr);
    else
      wgrad_kernel<false><<<grid, kWgThreads, 0, st>>>(N, K, R, rps, A, lda, nullptr, B, ldb, workspace,
                                                       row_sums ? wsb : nullptr);
  } else {
    (void)hipMemsetAsync(workspace, 0, sizeof(float) * (size_t)(N * K + N), st);
  }
  const int64_t c_blocks = (N * K / 4 + 63) / 64;
  const int64_t b_blocks = row_sums ? (N / 4 + 63) / 64 : 0;
  wgrad_reduce_kernel<<<(unsigned)(c_blocks + b_blocks), 1024, 0, st>>>(workspace, wsb, R > 0 ? splits : 1, N, K, C,
                                                                       ldc, row_sums, accumulate, c_blocks);
  return check_launch("rk_gemm_wgrad");
}
