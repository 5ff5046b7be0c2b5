// Fused dense layer on FP32 MFMA (v_mfma_f32_32x32x2_f32, exact f32 fma chain):
//   Y = epilogue(X . W^T)  with X [M, K] (row stride ldx), W [N, K] (nn.Linear layout).
//
// Tiling: 256-thread workgroup = 2x2 waves; each wave owns TM x TN tiles of 32x32, so the
// workgroup tile is (64*TM) x (64*TN).  K is staged through LDS in steps of 32; inside a
// step each lane reads a float4 of its A row and its W row (k = 8c + 4*(lane>>5) + comp)
// and issues 4 MFMAs, one per component — the k order is permuted, the sum is the same.
// LDS rows are padded to 36 floats, which makes the ds_read_b128 pattern conflict-free.
//
// Row epilogues (LayerNorm, pooling over row groups, the final Linear(N,1)+sigmoid head)
// need the whole row in one workgroup: those launches use one N tile (N <= 256) and pass
// the finished tile through LDS.
//
// Reference layers covered (reference snapshot): dcn.py:144-152,175-180;
// deepfm.py:100-112,143-151; din.py:26-36,272-285,312-316; deepcrossing.py:25-42,161-162;
// bst.py:59-64,73-75,86-90,203-214,238-247.
#include "common.h"

namespace rk {

constexpr int kBK = 32;
constexpr int kLDK = kBK + 4;

__device__ __forceinline__ float apply_act(const rk_epilogue& ep, float z, int n) {
  switch (ep.act) {
    case RK_ACT_RELU:
      return z < 0.f ? 0.f : z;  // keeps NaN, like torch.relu
    case RK_ACT_LEAKY:
      return z > 0.f ? z : z * ep.slope;
    case RK_ACT_DICE: {
      const float xn = z * ep.act_scale[n] + ep.act_shift[n];  // BatchNorm1d(affine=False), eval
      const float p = 1.0f / (1.0f + expf(-xn));
      return ep.act_alpha[n] * (1.0f - p) * z + p * z;
    }
    case RK_ACT_PRELU: {
      const float a = ep.act_alpha[ep.act_alpha_len == 1 ? 0 : n];
      return z > 0.f ? z : a * z;
    }
    default:
      return z;
  }
}

__device__ __forceinline__ float epi_elem(const rk_epilogue& ep, float z, int64_t m, int n, int N) {
  if (ep.bias) z += ep.bias[n];
  if (ep.residual) {
    float r = ep.residual[m * ep.ld_residual + n];
    if (ep.residual_periodic) r = r + ep.residual_periodic[(m % ep.residual_period) * (int64_t)N + n];
    z = r + z;
  }
  if (ep.pre_scale) z = z * ep.pre_scale[n] + ep.pre_shift[n];
  z = apply_act(ep, z, n);
  if (ep.post_scale) z = z * ep.post_scale[n] + ep.post_shift[n];
  return z;
}

template <int TM, int TN, bool VEC, bool ROWEPI>
__global__ __launch_bounds__(256) void linear_kernel(const float* __restrict__ X, int64_t ldx,
                                                     const float* __restrict__ Xp, int xperiod,
                                                     const float* __restrict__ W, int64_t ldw, int64_t M, int N,
                                                     int K, rk_epilogue ep, float* __restrict__ Y, int64_t ldy,
                                                     int rows_per_tile) {
  constexpr int BM = 64 * TM, BN = 64 * TN;
  constexpr int kStage = (BM + BN) * kLDK;
  constexpr int kTile = ROWEPI ? BM * (BN + 1) : 0;
  constexpr int kSmem = kStage > kTile ? kStage : kTile;
  __shared__ __attribute__((aligned(16))) float smem[kSmem];
  float* As = smem;
  float* Ws = smem + BM * kLDK;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hk = 4 * (lane >> 5);
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * rows_per_tile;
  const int rows = (int)min<int64_t>(min<int64_t>(rows_per_tile, BM), M - m0);
  const int n0 = blockIdx.y * BN;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  for (int k0 = 0; k0 < K; k0 += kBK) {
    if constexpr (VEC) {
      for (int i = tid; i < BM * (kBK / 4); i += 256) {
        const int r = i >> 3, c = (i & 7) * 4;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (r < rows && k0 + c < K) {
          const int64_t m = m0 + r;
          v = *reinterpret_cast<const f32x4*>(X + m * ldx + k0 + c);
          if (Xp) v += *reinterpret_cast<const f32x4*>(Xp + (m % xperiod) * (int64_t)K + k0 + c);
        }
        *reinterpret_cast<f32x4*>(As + r * kLDK + c) = v;
      }
      for (int i = tid; i < BN * (kBK / 4); i += 256) {
        const int r = i >> 3, c = (i & 7) * 4;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (n0 + r < N && k0 + c < K) v = *reinterpret_cast<const f32x4*>(W + (int64_t)(n0 + r) * ldw + k0 + c);
        *reinterpret_cast<f32x4*>(Ws + r * kLDK + c) = v;
      }
    } else {
      for (int i = tid; i < BM * kBK; i += 256) {
        const int r = i / kBK, c = i % kBK;
        float v = 0.f;
        if (r < rows && k0 + c < K) {
          const int64_t m = m0 + r;
          v = X[m * ldx + k0 + c];
          if (Xp) v += Xp[(m % xperiod) * (int64_t)K + k0 + c];
        }
        As[r * kLDK + c] = v;
      }
      for (int i = tid; i < BN * kBK; i += 256) {
        const int r = i / kBK, c = i % kBK;
        float v = 0.f;
        if (n0 + r < N && k0 + c < K) v = W[(int64_t)(n0 + r) * ldw + k0 + c];
        Ws[r * kLDK + c] = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 8) {
      f32x4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[i] = *reinterpret_cast<const f32x4*>(As + (wm * 32 * TM + i * 32 + l32) * kLDK + kk + hk);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[j] = *reinterpret_cast<const f32x4*>(Ws + (wn * 32 * TN + j * 32 + l32) * kLDK + kk + hk);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(a[i][c], b[j][c], acc[i][j]);
    }
    __syncthreads();
  }

  if constexpr (!ROWEPI) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * 32 * TN + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lr = wm * 32 * TM + i * 32 + acc_row(r, lane);
          if (lr < rows && n < N) {
            const int64_t m = m0 + lr;
            Y[m * ldy + n] = epi_elem(ep, acc[i][j][r], m, n, N);
          }
        }
      }
  } else {
    // 1) element-wise epilogue into the LDS tile [BM][BN+1]
    constexpr int LDT = BN + 1;
    float* T = smem;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wn * 32 * TN + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lr = wm * 32 * TM + i * 32 + acc_row(r, lane);
          float v = 0.f;
          if (lr < rows && n < N) v = epi_elem(ep, acc[i][j][r], m0 + lr, n, N);
          T[lr * LDT + n] = v;
        }
      }
    __syncthreads();
    // 2) per-row work: wave w takes rows w, w+4, ...; lane owns columns lane + 64*c
    constexpr int CPL = BN / 64;
    const float inv_n = 1.0f / (float)N;
    for (int lr = wave; lr < rows; lr += 4) {
      const int64_t m = m0 + lr;
      float v[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) v[c] = T[lr * LDT + lane + 64 * c];
      if (ep.has_ln) {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < CPL; ++c)
          if (lane + 64 * c < N) s += v[c];
        const float mean = wave_sum(s) * inv_n;
        float q = 0.f;
#pragma unroll
        for (int c = 0; c < CPL; ++c)
          if (lane + 64 * c < N) {
            const float d = v[c] - mean;
            q = fmaf(d, d, q);
          }
        const float rstd = 1.0f / sqrtf(wave_sum(q) * inv_n + ep.ln_eps);
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int n = lane + 64 * c;
          if (n < N) v[c] = (v[c] - mean) * rstd * ep.ln_gamma[n] + ep.ln_beta[n];
        }
      }
      if (Y) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int n = lane + 64 * c;
          if (n < N) Y[m * ldy + n] = v[c];
        }
      }
      if (ep.pool_out) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) T[lr * LDT + lane + 64 * c] = v[c];
      }
      if (ep.head_w) {
        float p = 0.f;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int n = lane + 64 * c;
          if (n < N) p = fmaf(v[c], ep.head_w[n], p);
        }
        p = wave_sum(p);
        if (lane == 0) {
          float logit = p + ep.head_b[0];
          if (ep.head_partial) logit = ep.head_partial[m] + logit;
          if (ep.fm1) {
            if (ep.head_aux) ep.head_aux[m] = logit;
            // final_layer(cat[fm1, fm2, deep]) — nn.Linear(3, 1)
            logit = ep.fm1[m] * ep.final_w[0] + ep.fm2[m] * ep.final_w[1] + logit * ep.final_w[2] + ep.final_b[0];
          }
          if (ep.head_logit) ep.head_logit[m] = logit;
          if (ep.head_prob) ep.head_prob[m] = 1.0f / (1.0f + expf(-logit));
        }
      }
    }
    if (ep.pool_out) {
      __syncthreads();
      const int64_t g = blockIdx.x;
      for (int n = tid; n < N; n += 256) {
        float s = 0.f;
        for (int lr = 0; lr < rows; ++lr) s += T[lr * LDT + n];
        if (ep.pool_mean) s = s / (float)ep.pool_len[g];
        ep.pool_out[g * ep.ld_pool + n] = s;
      }
    }
  }
}


template <int TM, int TN, bool ROWEPI>
static void launch(bool vec, dim3 grid, hipStream_t st, const float* X, int64_t ldx, const float* Xp, int xperiod,
                   const float* W, int64_t ldw, int64_t M, int N, int K, const rk_epilogue& ep, float* Y, int64_t ldy,
                   int rpt) {
  if (vec)
    linear_kernel<TM, TN, true, ROWEPI><<<grid, 256, 0, st>>>(X, ldx, Xp, xperiod, W, ldw, M, N, K, ep, Y, ldy, rpt);
  else
    linear_kernel<TM, TN, false, ROWEPI><<<grid, 256, 0, st>>>(X, ldx, Xp, xperiod, W, ldw, M, N, K, ep, Y, ldy, rpt);
}

}  // namespace rk

using namespace rk;

RK_API int rk_linear(const float* x, int64_t ldx, const float* x_periodic, int32_t x_period, const float* w,
                     int64_t ldw, int64_t M, int32_t N, int32_t K, const rk_epilogue* ep_in, float* y, int64_t ldy,
                     void* stream) {
  if (M < 0 || N <= 0 || K <= 0 || !x || !w || ldx < K || ldw < K)
    return fail(RK_ERR_INVALID, "rk_linear: bad shape M=%lld N=%d K=%d ldx=%lld ldw=%lld", (long long)M, N, K,
                (long long)ldx, (long long)ldw);
  if (x_periodic && x_period <= 0) return fail(RK_ERR_INVALID, "rk_linear: x_period must be > 0");
  rk_epilogue ep = {};
  if (ep_in) ep = *ep_in;
  const bool rowepi = ep.has_ln || ep.pool_out || ep.head_w;
  if (!rowepi && !y) return fail(RK_ERR_INVALID, "rk_linear: null output");
  if (y && ldy < N) return fail(RK_ERR_INVALID, "rk_linear: ldy < N");
  if (ep.residual && ep.ld_residual < N) return fail(RK_ERR_INVALID, "rk_linear: ld_residual < N");
  if (ep.residual_periodic && (!ep.residual || ep.residual_period <= 0))
    return fail(RK_ERR_INVALID, "rk_linear: residual_periodic needs residual and period > 0");
  if ((ep.pre_scale != nullptr) != (ep.pre_shift != nullptr) || (ep.post_scale != nullptr) != (ep.post_shift != nullptr))
    return fail(RK_ERR_INVALID, "rk_linear: affine scale/shift must come in pairs");
  if (ep.act == RK_ACT_DICE && (!ep.act_scale || !ep.act_shift || !ep.act_alpha))
    return fail(RK_ERR_INVALID, "rk_linear: Dice needs act_scale/act_shift/act_alpha");
  if (ep.act == RK_ACT_PRELU && (!ep.act_alpha || (ep.act_alpha_len != 1 && ep.act_alpha_len != N)))
    return fail(RK_ERR_INVALID, "rk_linear: PReLU needs act_alpha of length 1 or N");
  if (ep.act < 0 || ep.act > RK_ACT_PRELU) return fail(RK_ERR_INVALID, "rk_linear: unknown activation %d", ep.act);
  if (ep.has_ln && (!ep.ln_gamma || !ep.ln_beta)) return fail(RK_ERR_INVALID, "rk_linear: LayerNorm needs gamma/beta");
  if (ep.head_w && !ep.head_b) return fail(RK_ERR_INVALID, "rk_linear: head needs head_b");
  if (ep.fm1 && (!ep.fm2 || !ep.final_w || !ep.final_b)) return fail(RK_ERR_INVALID, "rk_linear: FM combine incomplete");
  if (M == 0) return RK_OK;
  const bool vec = (K % 4 == 0) && (ldx % 4 == 0) && (ldw % 4 == 0) && aligned16(x) && aligned16(w) &&
                   (!x_periodic || aligned16(x_periodic));
  hipStream_t st = (hipStream_t)stream;
  if (rowepi) {
    if (N > 256) return fail(RK_ERR_UNSUPPORTED, "rk_linear: row epilogue needs N <= 256 (N=%d)", N);
    int rpt = 64;
    if (ep.pool_out) {
      if (ep.pool_rows <= 0 || ep.pool_rows > 64 || M % ep.pool_rows != 0)
        return fail(RK_ERR_UNSUPPORTED, "rk_linear: pool_rows %d must divide M and be <= 64", ep.pool_rows);
      if (ep.pool_mean && !ep.pool_len) return fail(RK_ERR_INVALID, "rk_linear: mean pooling needs pool_len");
      rpt = ep.pool_rows;
    }
    const int64_t tiles = (M + rpt - 1) / rpt;
    if (tiles > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_linear: M too large");
    dim3 grid((unsigned)tiles, 1);
    if (N <= 64)
      launch<1, 1, true>(vec, grid, st, x, ldx, x_periodic, x_period, w, ldw, M, N, K, ep, y, ldy, rpt);
    else if (N <= 128)
      launch<1, 2, true>(vec, grid, st, x, ldx, x_periodic, x_period, w, ldw, M, N, K, ep, y, ldy, rpt);
    else
      launch<1, 4, true>(vec, grid, st, x, ldx, x_periodic, x_period, w, ldw, M, N, K, ep, y, ldy, rpt);
  } else {
    if (gemm_rows_try(x, ldx, nullptr, x_periodic, x_period, w, ldw, 0, M, N, K, y, ldy, 0, &ep, st))
      return check_launch("rk_linear");
    const int64_t big_tiles = ((M + 127) / 128) * ((N + 127) / 128);
    if (big_tiles >= 2 * num_cus()) {
      dim3 grid((unsigned)((M + 127) / 128), (unsigned)((N + 127) / 128));
      launch<2, 2, false>(vec, grid, st, x, ldx, x_periodic, x_period, w, ldw, M, N, K, ep, y, ldy, 128);
    } else {
      dim3 grid((unsigned)((M + 63) / 64), (unsigned)((N + 63) / 64));
      launch<1, 1, false>(vec, grid, st, x, ldx, x_periodic, x_period, w, ldw, M, N, K, ep, y, ldy, 64);
    }
  }
  return check_launch("rk_linear");
}
