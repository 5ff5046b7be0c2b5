// Fused-MLP machinery shared by rk_mlp_forward (mlp.hip) and the fused DIN forward (din_fused.hip).
//
// 16 rows per workgroup of 16 waves (4 per SIMD).  Activations live in two LDS buffers; each
// layer reads one and writes the other.  Layer math is FP32 MFMA v_mfma_f32_16x16x4_f32 (exact
// f32): wave w owns output tiles w and w+16 (16 columns each).  Per 16-deep K chunk a lane reads
// one float4 of its A row from LDS (k = 16c + 4*(lane>>4) + e) and one float4 of its weight row
// per tile from global memory, then issues 4 MFMAs per tile.  Weights are pre-packed
// (rk_mlp_pack_weight: rows padded to 64 columns, K padded to 64, zero fill), so every weight
// load is an unconditional aligned float4 and the chunk count is a multiple of the 4-deep
// register prefetch ring; weights stay L2-resident across the workgroups.
#pragma once

#include "common.h"

namespace rk {

constexpr int kMlpRows = 16;
constexpr int kMlpWaves = 16;
constexpr int kMlpThreads = 64 * kMlpWaves;
constexpr int kMlpPD = 4;    // prefetch depth (chunks)
constexpr int kMlpPad = 64;  // K and N padding of packed weights
constexpr int kMlpMaxN = 512;

typedef float f32x4_t __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int pad64(int v) { return (v + kMlpPad - 1) / kMlpPad * kMlpPad; }

__device__ __forceinline__ f32x4_t mfma16(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float layer_act(const rk_mlp_layer& L, float z, int n) {
  switch (L.act) {
    case RK_ACT_RELU:
      return z < 0.f ? 0.f : z;
    case RK_ACT_LEAKY:
      return z > 0.f ? z : z * L.slope;
    case RK_ACT_DICE: {
      const float xn = z * L.act_scale[n] + L.act_shift[n];
      const float p = 1.0f / (1.0f + expf(-xn));
      return L.act_alpha[n] * (1.0f - p) * z + p * z;
    }
    case RK_ACT_PRELU: {
      const float a = L.act_alpha[L.act_alpha_len == 1 ? 0 : n];
      return z > 0.f ? z : a * z;
    }
    default:
      return z;
  }
}

// One layer for a wave owning TPW tiles (t = wave + 16*j).
template <int TPW>
__device__ __forceinline__ void mlp_layer(const rk_mlp_layer& L, const float* __restrict__ in, int ldin,
                                          float* __restrict__ out, int ldout, int Kp, int wave, int lane) {
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const int kchunks = Kp / 16;  // multiple of kMlpPD
  const int64_t ldw = L.ldw;
  const float* wrow[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) wrow[j] = L.w + (int64_t)(16 * (wave + kMlpWaves * j) + li) * ldw + kq;

  f32x4_t acc[TPW];
  f32x4_t ring[kMlpPD][TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < kMlpPD; ++s)
#pragma unroll
    for (int j = 0; j < TPW; ++j) ring[s][j] = *reinterpret_cast<const f32x4_t*>(wrow[j] + 16 * s);

  const float* arow = in + li * ldin + kq;
  for (int c0 = 0; c0 < kchunks; c0 += kMlpPD) {
#pragma unroll
    for (int s = 0; s < kMlpPD; ++s) {
      const int c = c0 + s;
      const f32x4_t av = *reinterpret_cast<const f32x4_t*>(arow + 16 * c);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < TPW; ++j) acc[j] = mfma16(av[e], ring[s][j][e], acc[j]);
      // refill this slot with chunk c + PD (clamped: the tail re-reads the last chunk, unused)
      const int cn = min(c + kMlpPD, kchunks - 1);
#pragma unroll
      for (int j = 0; j < TPW; ++j) ring[s][j] = *reinterpret_cast<const f32x4_t*>(wrow[j] + 16 * cn);
      // keep the refill here: sinking it to the end of the unrolled body would leave each
      // slot's latency uncovered by the other slots' MFMAs
      __builtin_amdgcn_sched_barrier(0);
    }
  }

#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int n = 16 * (wave + kMlpWaves * j) + li;
    const bool real = n < L.n;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = (lane >> 4) * 4 + r;
      float z = 0.f;
      if (real) {
        z = acc[j][r];
        if (L.bias) z += L.bias[n];
        // x + f(x): the previous layer's input still sits in `out` (read-then-write, same lane)
        if (L.residual) z = out[row * ldout + n] + z;
        if (L.pre_scale) z = z * L.pre_scale[n] + L.pre_shift[n];
        z = layer_act(L, z, n);
        if (L.post_scale) z = z * L.post_scale[n] + L.post_shift[n];
      }
      out[row * ldout + n] = z;  // padded columns [n, Np) become the next layer's zero K pad
    }
  }
}

// Runs layers[0..nl) on the 16 rows staged (zero-padded to pad64(K0) columns) in buf0, then the
// head (one wave per row) or a plain copy of the last activation to y.  Must be called by all
// kMlpThreads threads of the workgroup.
__device__ __forceinline__ void mlp_rows(const rk_mlp_layer* __restrict__ layers, int nl, int K0, float* buf0,
                                         int ld0, float* buf1, int ld1, int64_t m0, int rows,
                                         const rk_epilogue& h, float* y, int64_t ldy, int tid) {
  const int lane = tid & 63, wave = tid >> 6;
  int Kp = pad64(K0);
  for (int l = 0; l < nl; ++l) {
    const rk_mlp_layer& L = layers[l];
    const int ntiles = pad64(L.n) / 16;  // multiple of 4
    const float* in = (l & 1) ? buf1 : buf0;
    float* out = (l & 1) ? buf0 : buf1;
    const int ldin = (l & 1) ? ld1 : ld0, ldout = (l & 1) ? ld0 : ld1;
    if (wave + kMlpWaves < ntiles) {
      mlp_layer<2>(L, in, ldin, out, ldout, Kp, wave, lane);
    } else if (wave < ntiles) {
      mlp_layer<1>(L, in, ldin, out, ldout, Kp, wave, lane);
    }
    __syncthreads();
    Kp = pad64(L.n);
  }
  const float* fin = (nl & 1) ? buf1 : buf0;
  const int ldf = (nl & 1) ? ld1 : ld0;
  const int K = nl ? layers[nl - 1].n : K0;
  if (h.head_w) {
    if (wave < rows) {
      const int r = wave;
      float p = 0.f;
      for (int n = lane; n < K; n += 64) p = fmaf(fin[r * ldf + n], h.head_w[n], p);
      p = wave_sum(p);
      if (lane == 0) {
        const int64_t m = m0 + r;
        float logit = p + h.head_b[0];
        if (h.head_partial) logit = h.head_partial[m] + logit;
        if (h.fm1) {
          if (h.head_aux) h.head_aux[m] = logit;
          logit = h.fm1[m] * h.final_w[0] + h.fm2[m] * h.final_w[1] + logit * h.final_w[2] + h.final_b[0];
        }
        if (h.head_logit) h.head_logit[m] = logit;
        if (h.head_prob) h.head_prob[m] = 1.0f / (1.0f + expf(-logit));
      }
    }
  } else if (y) {
    for (int i = tid; i < rows * K; i += kMlpThreads) {
      const int r = i / K, n = i % K;
      y[(m0 + r) * ldy + n] = fin[r * ldf + n];
    }
  }
}

// Host: validates a layer stack for mlp_rows and returns the two LDS buffer widths (floats,
// multiples of 64) needed by an input of width K0.
int mlp_validate(const rk_mlp_layer* layers, int nlayers, int K0, const rk_epilogue& head, int* need0, int* need1,
                 const char* what);

}  // namespace rk
