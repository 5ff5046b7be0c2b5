// Shared device/host helpers for the rankops HIP library (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/rankops.h"

#define RK_API extern "C" __attribute__((visibility("default")))

namespace rk {

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// 16-B alignment of a device pointer (float4 / dwordx4 paths are chosen on the host).
inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// ---- host-side error plumbing (runtime.cpp) ----
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);
// Device flag word of the current device (allocated by rk_init; may be null).
uint32_t* device_flags();
// Number of CUs on the current device (cached).
int num_cus();
// Raises `kern`'s dynamic-LDS limit to `bytes` on the current device, once per (kernel, device);
// thread-safe (runtime.hip).
void raise_lds_limit(const void* kern, int bytes);
// out[0] = scale * (sum of part[0..n)) / rows, one wave, fixed order (embedding.hip).
int launch_l2_final(const float* part, int n, int64_t rows, float scale, float* out, hipStream_t st);

// Tall-skinny FP32-MFMA GEMM (gemm_rows.hip); returns false when the shape is not its case.
bool gemm_rows_try(const float* A, int64_t lda, const float* A_mask, const float* Ap, int aperiod, const float* B,
                   int64_t ldb, int b_trans, int64_t M, int N, int K, float* C, int64_t ldc, int accumulate,
                   const rk_epilogue* ep, hipStream_t st);

// rk_bst_forward_blocks at d_model 16 (bst_small.hip)
int bst_small_forward(const float* table, int64_t table_rows, int64_t ld_table, const int64_t* seq, int64_t ld_seq,
                      int32_t T, const int64_t* seq_len, int64_t batch, int32_t heads, int32_t nblocks,
                      const float* const* block_params, const float* block_scalars, float* pool_out, int64_t ld_pool,
                      int32_t pool_mean, hipStream_t st);

// ---- device helpers ----
// Wave index of the calling thread in its workgroup, as a wave-uniform (SGPR) value: branches and
// addresses that depend only on it compile to scalar code.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// The same all-lane sum with the in-row steps on DPP (xor 1, xor 2 by quad_perm; 8- and 16-lane
// mirrors) and only the two cross-row steps through ds_bpermute: 4 VALU ops + 2 LDS round trips
// instead of 6.  Every step adds two partial sums that are equal in both lanes, so all lanes end
// with the same bits (a different association from wave_sum: the two are not interchangeable
// where results must match bit for bit).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f32<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f32<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f32<0x141>(v);  // row_half_mirror
  v += dpp_f32<0x140>(v);  // row_mirror
  v += __shfl_xor(v, 16, kWave);
  v += __shfl_xor(v, 32, kWave);
  return v;
}

// Sum / max over the 16 lanes of each DPP row, all on DPP (no LDS round trip).  The pairing is the
// xor butterfly's (1, 2, then the other quad, then the other half), so the result has exactly the
// bits of `for x in 1,2,4,8: v += __shfl_xor(v, x)`.
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f32<0xB1>(v);
  v += dpp_f32<0x4E>(v);
  v += dpp_f32<0x141>(v);
  v += dpp_f32<0x140>(v);
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f32<0xB1>(v));
  v = fmaxf(v, dpp_f32<0x4E>(v));
  v = fmaxf(v, dpp_f32<0x141>(v));
  v = fmaxf(v, dpp_f32<0x140>(v));
  return v;
}

// Sums of N values over the 16 lanes of each DPP row, transposed: each step pairs lanes across one
// lane bit (row_mirror: bit 3, row_half_mirror: bit 2, quad_perm [2,3,0,1]: bit 1, [1,0,3,2]: bit 0)
// and, while a lane still holds more than one value, keeps one half (the upper half where its bit is
// set) and adds the partner's copy of it — N - 1 + log2(16 / N) DPP moves instead of 4 N.  Lane p16
// returns the row sum of element e = (N/2) bit3 + (N/4) bit2 + (N/8) bit1, i.e. e = p16 / (16 / N);
// v is clobbered.  Deterministic (fixed pairing), not bit-equal to N row16_sum calls.
template <int CTRL, int BIT, int N>
__device__ __forceinline__ void row16_split_step(float* v, int p16) {
  const bool hi = (p16 >> BIT) & 1;
#pragma unroll
  for (int i = 0; i < N / 2; ++i) {
    const float keep = hi ? v[i + N / 2] : v[i];
    const float send = hi ? v[i] : v[i + N / 2];
    v[i] = keep + dpp_f32<CTRL>(send);
  }
}
template <int N>
__device__ __forceinline__ float row16_transpose_sum(float (&v)[N], int p16) {
  static_assert(N == 1 || N == 2 || N == 4 || N == 8, "1, 2, 4 or 8 values");
  if constexpr (N >= 2) row16_split_step<0x140, 3, N>(v, p16);
  else v[0] += dpp_f32<0x140>(v[0]);
  if constexpr (N >= 4) row16_split_step<0x141, 2, N / 2>(v, p16);
  else v[0] += dpp_f32<0x141>(v[0]);
  if constexpr (N >= 8) row16_split_step<0x4E, 1, N / 4>(v, p16);
  else v[0] += dpp_f32<0x4E>(v[0]);
  v[0] += dpp_f32<0xB1>(v[0]);
  return v[0];
}

// Sums across lane bit 4 / bit 5 on the gfx950 cross-row swaps (VALU, no LDS round trip):
// v_permlane16_swap / v_permlane32_swap with vdst = vsrc = v leave v of the partner row / half in
// one of the two results and v in the other, in the same (low lane, high lane) order in both lanes
// of a pair, so r[0] + r[1] is bit-identical to v + __shfl_xor(v, 16 | 32) in every lane.
__device__ __forceinline__ float xor16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Sum over the 32 lanes of each half-wave (lanes l and l^32 are not combined).
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.0f / (1.0f + expf(-x)); }
// Sigmoid on the transcendental unit: v_exp_f32 (2^x) and v_rcp_f32, each ~1 ulp, 4 instructions
// instead of the ~25 of expf + an IEEE divide; saturates to exactly 0 / 1 where the reference
// formula does.  Used in the hot eval epilogues (Dice); relative error ~1e-7 against 1e-4 parity.
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896341f));
}

__device__ __forceinline__ void flag_oob(uint32_t* flags) {
  if (flags) atomicOr(flags, RK_FLAG_INDEX_OOB);
}

// Reads table row `idx` (bounds-checked): returns nullptr for an out-of-range index.
__device__ __forceinline__ const float* table_row(const rk_segment& s, int64_t b,
                                                  uint32_t* flags) {
  const int64_t r = s.idx[b * s.idx_stride];
  if (r < 0 || r >= s.rows) {
    flag_oob(flags);
    return nullptr;
  }
  return s.src + r * s.src_ld;
}

// Row of a segment for sample b (table or dense); nullptr if OOB.
__device__ __forceinline__ const float* segment_row(const rk_segment& s, int64_t b,
                                                    uint32_t* flags) {
  if (s.idx) return table_row(s, b, flags);
  return s.src + b * s.src_ld;
}

// FP32-input MFMA, 32x32x2: lane l supplies A[l&31][l>>5] and B[l>>5][l&31];
// accumulator register r of lane l is D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31].
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int r, int lane) {
  return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}

// Segment table passed by value as a kernel argument.
struct SegTable {
  rk_segment s[RK_MAX_SEGMENTS];
};

}  // namespace rk
