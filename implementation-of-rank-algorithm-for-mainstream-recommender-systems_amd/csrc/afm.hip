// AFM forward, fully fused (reference: AFM.forward, afm.py:92-119).
//
//   dense_logit = dense . w_d + b_d                                     afm.py:94
//   pair[p]     = e_i * e_j   for i < j in field order                  afm.py:101-108
//   score[p]    = h . relu(W_a pair[p] + b_a) + b_h                     afm.py:110
//   w           = softmax_p(score)                                      afm.py:111
//   logit       = dense_logit + p_w . sum_p w[p] pair[p] + p_b          afm.py:113-117
//
// One wave per sample.  The field embeddings of the wave's sample are staged in LDS; lane a
// owns attention units a, a+64, ... (their W_a rows live in registers) and accumulates its
// share of every pair score; one wave reduction per pair finishes the score.
#include <cstdlib>

#include "common.h"
#include "mlp_core.h"

namespace rk {

constexpr int kAfmMaxFields = 16;
constexpr int kAfmMaxDim = 64;
constexpr int kAfmMaxUnitsPerLane = 4;  // attention factor <= 256
constexpr int kAfmMaxPairs = kAfmMaxFields * (kAfmMaxFields - 1) / 2;

struct AfmFields {
  rk_segment s[kAfmMaxFields];
};

template <int D, int UPL>
__global__ __launch_bounds__(256) void afm_kernel(AfmFields fields, int F, int64_t batch,
                                                  const float* __restrict__ dense, int64_t ld_dense, int nd,
                                                  const float* __restrict__ dense_w, const float* __restrict__ dense_b,
                                                  const float* __restrict__ att_w, const float* __restrict__ att_b,
                                                  int A, const float* __restrict__ att_h,
                                                  const float* __restrict__ att_hb, const float* __restrict__ p_w,
                                                  const float* __restrict__ p_b, float* __restrict__ logit_out,
                                                  float* __restrict__ prob_out, uint32_t* flags) {
  __shared__ float emb[4][kAfmMaxFields * D];
  __shared__ float score[4][kAfmMaxPairs];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* e = emb[wave];
  float* sc = score[wave];

  // lane-resident attention weights
  float wa[UPL][D];
  float ba[UPL], ha[UPL];
#pragma unroll
  for (int u = 0; u < UPL; ++u) {
    const int a = lane + 64 * u;
    const bool on = a < A;
#pragma unroll
    for (int d = 0; d < D; ++d) wa[u][d] = on ? att_w[(int64_t)a * D + d] : 0.f;
    ba[u] = on ? att_b[a] : 0.f;
    ha[u] = on ? att_h[a] : 0.f;
  }
  const int P = F * (F - 1) / 2;

  for (int64_t b = (int64_t)blockIdx.x * 4 + wave; b < batch; b += (int64_t)gridDim.x * 4) {
    for (int i = lane; i < F * D; i += 64) {
      const int f = i / D, d = i % D;
      const float* row = segment_row(fields.s[f], b, flags);
      e[i] = row ? row[d] : 0.f;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();

    int p = 0;
    for (int i = 0; i < F; ++i)
      for (int j = i + 1; j < F; ++j, ++p) {
        float pr[D];
#pragma unroll
        for (int d = 0; d < D; ++d) pr[d] = e[i * D + d] * e[j * D + d];
        float part = 0.f;
#pragma unroll
        for (int u = 0; u < UPL; ++u) {
          float z = ba[u];
          // nn.Linear(D, A): sum_d pair[d] * W[a][d] + b[a]
          float acc = 0.f;
#pragma unroll
          for (int d = 0; d < D; ++d) acc = fmaf(pr[d], wa[u][d], acc);
          z = acc + z;
          z = z < 0.f ? 0.f : z;
          part = fmaf(z, ha[u], part);
        }
        part = wave_sum(part) + att_hb[0];
        if (lane == 0) sc[p] = part;
      }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();

    // softmax over pairs (every lane computes the same weights)
    float mx = -INFINITY;
    for (int q = 0; q < P; ++q) mx = fmaxf(mx, sc[q]);
    float den = 0.f;
    for (int q = 0; q < P; ++q) den += expf(sc[q] - mx);

    // weighted pair sum: lane d < D owns component d
    float ws = 0.f;
    if (lane < D) {
      int q = 0;
      for (int i = 0; i < F; ++i)
        for (int j = i + 1; j < F; ++j, ++q) {
          const float w = expf(sc[q] - mx) / den;
          ws += (e[i * D + lane] * e[j * D + lane]) * w;
        }
    }
    float afm = wave_sum(lane < D ? ws * p_w[lane] : 0.f) + p_b[0];
    float dl = 0.f;
    for (int k = lane; k < nd; k += 64) dl = fmaf(dense[b * ld_dense + k], dense_w[k], dl);
    dl = wave_sum(dl) + dense_b[0];
    if (lane == 0) {
      const float t = dl + afm;
      logit_out[b] = t;
      prob_out[b] = 1.0f / (1.0f + expf(-t));
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
  }
}

// The same forward with the attention MLP on the matrix cores (round 5): per sample the pair
// products form a [P x D] matrix and the attention layer is [P x D] . W_a^T ([D x A]) — P = 28 pairs,
// D = 8, A = 128 at afm.py's defaults — so one wave runs it as ceil(P/16) x NT tiles of
// v_mfma_f32_16x16x4_f32 over D/4 K-steps: lane l feeds pair 16 mt + l % 16, dims 4 s + l / 16 (the
// A operand, products formed from the LDS-staged embeddings) and holds W_a's fragments (the B
// operand: unit 16 t + l % 16, dims 4 s + l / 16) in registers for the whole launch.  Each output
// register is relu(. + b_a) * h, summed over the lane's unit tiles, then over the row's 16 units
// (row16_transpose_sum): the pair scores.  Softmax and the weighted sum run one pair per lane:
// afm = sum_p w_p (pair_p . p_w) + p_b, the weighted pair vector contracted with p first (the same
// value as p(sum_p w_p pair_p), reassociated).  KS = D / 4 (D in {4, 8, 16}), NT = unit tiles of 16
// (A <= 128, rounded up to 2 / 4 / 8: the extra units have zero weights).
constexpr int kAfmMfmaMaxPairs = 120;  // F <= 16
template <int KS, int NT>
__global__ __launch_bounds__(256) void afm_mfma_kernel(AfmFields fields, int F, int64_t batch,
                                                       const float* __restrict__ dense, int64_t ld_dense, int nd,
                                                       const float* __restrict__ dense_w,
                                                       const float* __restrict__ dense_b,
                                                       const float* __restrict__ att_w, const float* __restrict__ att_b,
                                                       int A, const float* __restrict__ att_h,
                                                       const float* __restrict__ att_hb, const float* __restrict__ p_w,
                                                       const float* __restrict__ p_b, float* __restrict__ logit_out,
                                                       float* __restrict__ prob_out, uint32_t* flags) {
  constexpr int D = 4 * KS;
  __shared__ float emb[4][kAfmMaxFields * D];
  __shared__ float score[4][kAfmMfmaMaxPairs];
  __shared__ uint8_t pfi[kAfmMfmaMaxPairs], pfj[kAfmMfmaMaxPairs];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, p16 = lane & 15, grp = lane >> 4;
  float* e = emb[wave];
  float* sc = score[wave];
  const int P = F * (F - 1) / 2;
  // pair p -> (i, j), i < j in field order (afm.py:101-108)
  if ((int)threadIdx.x < P) {
    int p = threadIdx.x, i = 0;
    while (p >= F - 1 - i) {
      p -= F - 1 - i;
      ++i;
    }
    pfi[threadIdx.x] = (uint8_t)i;
    pfj[threadIdx.x] = (uint8_t)(i + 1 + p);
  }
  // W_a fragments, b_a and h of this lane's unit columns 16 t + p16
  float bw[NT][KS], ba[NT], hh[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int a = 16 * t + p16;
    const bool on = a < A;
#pragma unroll
    for (int s = 0; s < KS; ++s) bw[t][s] = on ? att_w[(int64_t)a * D + 4 * s + grp] : 0.f;
    ba[t] = on ? att_b[a] : 0.f;
    hh[t] = on ? att_h[a] : 0.f;
  }
  float pw[D];
#pragma unroll
  for (int d = 0; d < D; ++d) pw[d] = p_w[d];
  const float hb = att_hb[0], pb = p_b[0];
  __syncthreads();  // the pair tables
  const int MT = (P + 15) >> 4;

  for (int64_t b = (int64_t)blockIdx.x * 4 + wave; b < batch; b += (int64_t)gridDim.x * 4) {
    for (int i = lane; i < F * D; i += 64) {
      const int f = i / D, d = i % D;
      const float* row = segment_row(fields.s[f], b, flags);
      e[i] = row ? row[d] : 0.f;
    }
    float dl = 0.f;
    for (int k = lane; k < nd; k += 64) dl = fmaf(dense[b * ld_dense + k], dense_w[k], dl);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();

    for (int mt = 0; mt < kAfmMfmaMaxPairs / 16 + 1; ++mt) {
      if (mt >= MT) break;
      const int p = 16 * mt + p16;
      const bool pv = p < P;
      const int fi = pv ? pfi[p] : 0, fj = pv ? pfj[p] : 0;
      float a[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int d = 4 * s + grp;
        a[s] = pv ? e[fi * D + d] * e[fj * D + d] : 0.f;
      }
      f32x4_t acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) acc[t] = mfma16(a[s], bw[t][s], acc[t]);
      }
      // lane l, register r: pair 16 mt + 4 grp + r, unit 16 t + p16
      float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float z = acc[t][r] + ba[t];
          z = z < 0.f ? 0.f : z;  // relu (NaN propagates, as torch.relu)
          part[r] = fmaf(z, hh[t], part[r]);
        }
      const float sum = row16_transpose_sum<4>(part, p16);  // pair 16 mt + 4 grp + p16 / 4
      const int q = 16 * mt + 4 * grp + (p16 >> 2);
      if ((p16 & 3) == 0 && q < P) sc[q] = sum + hb;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();

    // softmax over the pairs and the contracted weighted sum, pairs lane and lane + 64
    float sp[2], tp[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = lane + 64 * k;
      const bool pv = p < P;
      sp[k] = pv ? sc[p] : -INFINITY;
      float t = 0.f;
      if (pv) {
        const int fi = pfi[p], fj = pfj[p];
#pragma unroll
        for (int d = 0; d < D; ++d) t = fmaf(e[fi * D + d] * e[fj * D + d], pw[d], t);
      }
      tp[k] = t;
    }
    const float mx = wave_max(fmaxf(sp[0], sp[1]));
    float ex[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) ex[k] = lane + 64 * k < P ? expf(sp[k] - mx) : 0.f;
    const float den = wave_sum(ex[0] + ex[1]);
    const float afm = wave_sum((ex[0] / den) * tp[0] + (ex[1] / den) * tp[1]) + pb;
    dl = wave_sum(dl) + dense_b[0];
    if (lane == 0) {
      const float t = dl + afm;
      logit_out[b] = t;
      prob_out[b] = 1.0f / (1.0f + expf(-t));
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
  }
}

// Round 6: the same forward with S samples per wave and their pair rows packed into shared MFMA
// tiles.  Per wave: lanes (s, f), s < S, f < F, load sample b0 + s's index of field f and its
// D-float row (float4s) — every load of the S samples issued before the one wait — and stage the
// rows in LDS; lanes s < S form the dense dot of sample b0 + s meanwhile.  The S x P pair rows
// (row r = s P + p) fill ceil(S P / 16) tiles of v_mfma_f32_16x16x4_f32 (7 fields, S = 2: 42 rows =
// 3 tiles, 88 % full, instead of 2 tiles at 66 % per sample), each tile NT independent accumulator
// chains of depth KS, the W_a fragments in registers as in afm_mfma_kernel.  Scores go to LDS; then
// LPS = 16 / 32 / 64 lanes per sample (P <= LPS) run the softmax and the contracted weighted sum
// with segment reductions on DPP and the cross-row permlane swaps.  One wait after the staging and
// one LDS hand-off per phase for all S samples (afm_mfma_kernel: two per sample, and one for the
// outputs' stores).  Same arithmetic per pair as afm_mfma_kernel; the per-sample sums run in a
// different (fixed) order.
constexpr int kAfmTileMaxRows = 256;  // S * P
template <int LPS>
__device__ __forceinline__ float seg_sum(float v) {
  v = row16_sum(v);
  if constexpr (LPS >= 32) v = xor16_sum(v);
  if constexpr (LPS >= 64) v = xor32_sum(v);
  return v;
}
template <int LPS>
__device__ __forceinline__ float seg_max(float v) {
  v = row16_max(v);
  if constexpr (LPS >= 32) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  if constexpr (LPS >= 64) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  return v;
}

// softmax + contracted weighted sum of the wave's S samples, LPS lanes per sample (P <= LPS)
template <int D, int S, int LPS>
__device__ __forceinline__ void afm_tiles_softmax(const float* e, const float* sc, const uint32_t* rinfo, int P,
                                                  int64_t b0, int64_t batch, float dl, float db, float pb,
                                                  const float (&pw)[D], float* __restrict__ logit_out,
                                                  float* __restrict__ prob_out) {
  constexpr int SPP = 64 / LPS;  // samples per pass
  const int lane = threadIdx.x & 63, sl = lane / LPS, p = lane % LPS;
#pragma unroll
  for (int s0 = 0; s0 < S; s0 += SPP) {
    const int s = s0 + sl;
    const bool v = s < S && p < P && b0 + s < batch;
    float scr = -INFINITY, tp = 0.f;
    if (v) {
      scr = sc[s * P + p];
      const uint32_t ri = rinfo[s * P + p];
      const int oi = (int)(ri & 0xffffu) * D, oj = (int)(ri >> 16) * D;
#pragma unroll
      for (int d = 0; d < D; ++d) tp = fmaf(e[oi + d] * e[oj + d], pw[d], tp);
    }
    const float mx = seg_max<LPS>(scr);
    const float ex = v ? expf(scr - mx) : 0.f;
    const float den = seg_sum<LPS>(ex);
    const float afm = seg_sum<LPS>(v ? (ex / den) * tp : 0.f) + pb;
    const float dls = __shfl(dl, s < S ? s : 0, kWave) + db;
    if (p == 0 && s < S && b0 + s < batch) {
      const float t = dls + afm;
      logit_out[b0 + s] = t;
      prob_out[b0 + s] = 1.0f / (1.0f + expf(-t));
    }
  }
}

template <int KS, int NT, int S>
__global__ __launch_bounds__(256) void afm_tiles_kernel(AfmFields fields, int F, int64_t batch,
                                                        const float* __restrict__ dense, int64_t ld_dense, int nd,
                                                        const float* __restrict__ dense_w,
                                                        const float* __restrict__ dense_b,
                                                        const float* __restrict__ att_w, const float* __restrict__ att_b,
                                                        int A, const float* __restrict__ att_h,
                                                        const float* __restrict__ att_hb, const float* __restrict__ p_w,
                                                        const float* __restrict__ p_b, float* __restrict__ logit_out,
                                                        float* __restrict__ prob_out, uint32_t* flags) {
  constexpr int D = 4 * KS;
  __shared__ __attribute__((aligned(16))) float emb[4][64 * D];  // S * F <= 64 staged rows per wave
  __shared__ float score[4][kAfmTileMaxRows];
  __shared__ uint32_t rinfo[kAfmTileMaxRows];  // pair row r -> staged rows (s F + i) | (s F + j) << 16
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, p16 = lane & 15, grp = lane >> 4;
  const int P = F * (F - 1) / 2, R = S * P;
  for (int r = threadIdx.x; r < R; r += 256) {
    const int s = r / P;
    int p = r - s * P, i = 0;
    while (p >= F - 1 - i) {  // pair p -> (i, j), i < j in field order (afm.py:101-108)
      p -= F - 1 - i;
      ++i;
    }
    rinfo[r] = (uint32_t)(s * F + i) | (uint32_t)(s * F + i + 1 + p) << 16;
  }
  const int64_t b0 = ((int64_t)blockIdx.x * 4 + wave) * S;
  float* e = emb[wave];
  float* sc = score[wave];
  // stage: lane (s, f) loads sample b0 + s's row of field f (all loads in flight together).  (A
  // field-by-field staging with the descriptors in scalar registers measured slower: the compiler
  // closes its per-field branches with waits on every load in flight, 14.6 vs 11.0 us at 4,096.)
  f32x4_t rv[KS];
  const int SF = S * F;
  {
    const float* row = nullptr;
    if (lane < SF) {
      const int s = lane / F, f = lane - s * F;
      const int64_t b = b0 + s;
      if (b < batch) row = segment_row(fields.s[f], b, flags);
    }
#pragma unroll
    for (int k = 0; k < KS; ++k)
      rv[k] = row ? *reinterpret_cast<const f32x4_t*>(row + 4 * k) : (f32x4_t){0.f, 0.f, 0.f, 0.f};
  }
  float dl = 0.f;
  if (lane < S && b0 + lane < batch) {
    const float* x = dense + (b0 + lane) * ld_dense;
    for (int k = 0; k < nd; ++k) dl = fmaf(x[k], dense_w[k], dl);
  }
  // W_a fragments, b_a and h of this lane's unit columns 16 t + p16 (as afm_mfma_kernel)
  float bw[NT][KS], ba[NT], hh[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int a = 16 * t + p16;
    const bool on = a < A;
#pragma unroll
    for (int s = 0; s < KS; ++s) bw[t][s] = on ? att_w[(int64_t)a * D + 4 * s + grp] : 0.f;
    ba[t] = on ? att_b[a] : 0.f;
    hh[t] = on ? att_h[a] : 0.f;
  }
  const float hb = att_hb[0], pb = p_b[0], db = dense_b[0];
  if (lane < SF) {
#pragma unroll
    for (int k = 0; k < KS; ++k) *reinterpret_cast<f32x4_t*>(e + lane * D + 4 * k) = rv[k];
  }
  __syncthreads();  // rinfo (whole workgroup) and this wave's staged rows
  if (b0 >= batch) return;
#if defined(RK_AFM_PHASE) && RK_AFM_PHASE == 1  // timing builds only (wrong outputs): staging only
  if (lane < S && b0 + lane < batch) logit_out[b0 + lane] = e[lane] + dl;
  return;
#endif

  // the pair tiles two at a time: both tiles' products, then their 2 NT independent accumulator
  // chains interleaved, then both epilogues — one wave per SIMD at 4,096 samples, so only a
  // wave's own independent work hides the MFMA and LDS latencies.  A second tile past MT reads as
  // zero rows and stores nothing (its rows are >= R); per-tile arithmetic as one tile at a time.
  const int MT = (R + 15) >> 4;
  auto tile_in = [&](int mt, float (&a)[KS]) {
    const int r = 16 * mt + p16;
    const bool rvld = r < R;
    const uint32_t ri = rvld ? rinfo[r] : 0u;
    const int oi = (int)(ri & 0xffffu) * D, oj = (int)(ri >> 16) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int d = 4 * s + grp;
      a[s] = rvld ? e[oi + d] * e[oj + d] : 0.f;
    }
  };
  auto tile_out = [&](int mt, const f32x4_t (&acc)[NT]) {
    float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float z = acc[t][q] + ba[t];
        z = z < 0.f ? 0.f : z;  // relu (NaN propagates, as torch.relu)
        part[q] = fmaf(z, hh[t], part[q]);
      }
    const float sum = row16_transpose_sum<4>(part, p16);  // pair row 16 mt + 4 grp + p16 / 4
    const int q = 16 * mt + 4 * grp + (p16 >> 2);
    if ((p16 & 3) == 0 && q < R) sc[q] = sum + hb;
  };
  for (int mt = 0; mt < MT; mt += 2) {
    float a0[KS], a1[KS];
    tile_in(mt, a0);
    tile_in(mt + 1, a1);
    f32x4_t acc0[NT], acc1[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      acc0[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      acc1[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        acc0[t] = mfma16(a0[s], bw[t][s], acc0[t]);
        acc1[t] = mfma16(a1[s], bw[t][s], acc1[t]);
      }
    }
    tile_out(mt, acc0);
    tile_out(mt + 1, acc1);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the scores are in LDS
  __builtin_amdgcn_wave_barrier();

#if defined(RK_AFM_PHASE) && RK_AFM_PHASE == 2  // timing builds only: staging + the pair-score MFMAs
  if (lane < S && b0 + lane < batch) logit_out[b0 + lane] = sc[lane] + dl;
  return;
#endif
  float pw[D];
#pragma unroll
  for (int d = 0; d < D; ++d) pw[d] = p_w[d];
  if (P <= 16)
    afm_tiles_softmax<D, S, 16>(e, sc, rinfo, P, b0, batch, dl, db, pb, pw, logit_out, prob_out);
  else if (P <= 32)
    afm_tiles_softmax<D, S, 32>(e, sc, rinfo, P, b0, batch, dl, db, pb, pw, logit_out, prob_out);
  else
    afm_tiles_softmax<D, S, 64>(e, sc, rinfo, P, b0, batch, dl, db, pb, pw, logit_out, prob_out);
}

}  // namespace rk

using namespace rk;

RK_API int rk_afm_forward(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch,
                          const float* dense, int64_t ld_dense, int32_t num_dense, const float* dense_w,
                          const float* dense_b, const float* att_w, const float* att_b, int32_t att_factor,
                          const float* att_h, const float* att_hb, const float* p_w, const float* p_b, float* logit,
                          float* prob, void* stream) {
  if (!fields || num_fields < 2 || num_fields > kAfmMaxFields)
    return fail(RK_ERR_UNSUPPORTED, "rk_afm_forward: %d fields (need 2..%d)", num_fields, kAfmMaxFields);
  if (att_factor <= 0 || att_factor > 64 * kAfmMaxUnitsPerLane)
    return fail(RK_ERR_UNSUPPORTED, "rk_afm_forward: attention factor %d > %d", att_factor, 64 * kAfmMaxUnitsPerLane);
  if (!att_w || !att_b || !att_h || !att_hb || !p_w || !p_b || !logit || !prob ||
      (num_dense > 0 && (!dense || !dense_w)) || !dense_b)
    return fail(RK_ERR_INVALID, "rk_afm_forward: null pointer");
  AfmFields t;
  for (int f = 0; f < num_fields; ++f) {
    if (!fields[f].src || fields[f].dim != dim) return fail(RK_ERR_INVALID, "rk_afm_forward: field %d dim mismatch", f);
    t.s[f] = fields[f];
  }
  for (int f = num_fields; f < kAfmMaxFields; ++f) t.s[f] = fields[num_fields - 1];  // afm_tiles_kernel's padding slots
  if (batch <= 0) return batch == 0 ? RK_OK : fail(RK_ERR_INVALID, "rk_afm_forward: negative batch");
  const unsigned blocks = (unsigned)std::min<int64_t>((batch + 3) / 4, (int64_t)num_cus() * 8);
  hipStream_t st = (hipStream_t)stream;
  uint32_t* fl = device_flags();
  static const bool mfma_on = [] {  // RANKOPS_AFM_MFMA=0: the VALU kernel (A/B)
    const char* e = getenv("RANKOPS_AFM_MFMA");
    return !(e && e[0] == '0');
  }();
  // samples per wave of afm_tiles_kernel (RANKOPS_AFM_S: 0 = afm_mfma_kernel, one sample per wave)
  const int tile_s = [] {  // read per call (tests switch it)
    const char* e = getenv("RANKOPS_AFM_S");
    const int v = e ? atoi(e) : 4;  // S = 4: 10.97 us at 4,096 (S = 2: 11.18, S = 0: 15.63), profiles/r06/afm_ab.log
    return v == 0 || v == 2 || v == 4 ? v : 4;
  }();
  const int P = num_fields * (num_fields - 1) / 2;
  bool rows16 = true;  // float4 row loads: 16-B aligned rows
  for (int f = 0; f < num_fields; ++f)
    rows16 = rows16 && aligned16(fields[f].src) && fields[f].src_ld % 4 == 0;
  if (mfma_on && tile_s && (dim == 4 || dim == 8 || dim == 16) && att_factor <= 128 && P <= 64 && rows16 &&
      tile_s * num_fields <= 64 && tile_s * P <= kAfmTileMaxRows) {
    const int nt = (att_factor + 15) / 16;
    const unsigned tblocks = (unsigned)((batch + 4 * tile_s - 1) / (4 * tile_s));
    auto go = [&](auto kern) {
      kern<<<tblocks, 256, 0, st>>>(t, num_fields, batch, dense, ld_dense, num_dense, dense_w, dense_b, att_w, att_b,
                                    att_factor, att_h, att_hb, p_w, p_b, logit, prob, fl);
    };
    auto by_s = [&](auto ks, auto ntc) {
      constexpr int KS = decltype(ks)::value, NT = decltype(ntc)::value;
      if (tile_s == 4)
        go(afm_tiles_kernel<KS, NT, 4>);
      else
        go(afm_tiles_kernel<KS, NT, 2>);
    };
    auto by_nt = [&](auto ks) {
      if (nt <= 2)
        by_s(ks, std::integral_constant<int, 2>{});
      else if (nt <= 4)
        by_s(ks, std::integral_constant<int, 4>{});
      else
        by_s(ks, std::integral_constant<int, 8>{});
    };
    if (dim == 4)
      by_nt(std::integral_constant<int, 1>{});
    else if (dim == 8)
      by_nt(std::integral_constant<int, 2>{});
    else
      by_nt(std::integral_constant<int, 4>{});
    return check_launch("rk_afm_forward");
  }
  if (mfma_on && (dim == 4 || dim == 8 || dim == 16) && att_factor <= 128) {
    const int nt = (att_factor + 15) / 16;
    auto go = [&](auto kern) {
      kern<<<blocks, 256, 0, st>>>(t, num_fields, batch, dense, ld_dense, num_dense, dense_w, dense_b, att_w, att_b,
                                   att_factor, att_h, att_hb, p_w, p_b, logit, prob, fl);
    };
    auto by_nt = [&](auto ks) {
      constexpr int KS = decltype(ks)::value;
      if (nt <= 2)
        go(afm_mfma_kernel<KS, 2>);
      else if (nt <= 4)
        go(afm_mfma_kernel<KS, 4>);
      else
        go(afm_mfma_kernel<KS, 8>);
    };
    if (dim == 4)
      by_nt(std::integral_constant<int, 1>{});
    else if (dim == 8)
      by_nt(std::integral_constant<int, 2>{});
    else
      by_nt(std::integral_constant<int, 4>{});
    return check_launch("rk_afm_forward");
  }
  const int upl = (att_factor + 63) / 64;
#define RK_AFM_LAUNCH(DD, UU)                                                                                    \
  afm_kernel<DD, UU><<<blocks, 256, 0, st>>>(t, num_fields, batch, dense, ld_dense, num_dense, dense_w, dense_b, \
                                             att_w, att_b, att_factor, att_h, att_hb, p_w, p_b, logit, prob, fl)
#define RK_AFM_CASE(DD)              \
  case DD:                           \
    if (upl == 1)                    \
      RK_AFM_LAUNCH(DD, 1);          \
    else if (upl == 2)               \
      RK_AFM_LAUNCH(DD, 2);          \
    else                             \
      RK_AFM_LAUNCH(DD, 4);          \
    break;
  switch (dim) {
    RK_AFM_CASE(4)
    RK_AFM_CASE(8)
    RK_AFM_CASE(16)
    RK_AFM_CASE(32)
    default:
      return fail(RK_ERR_UNSUPPORTED, "rk_afm_forward: embedding dim %d not in {4,8,16,32}", dim);
  }
#undef RK_AFM_CASE
#undef RK_AFM_LAUNCH
  return check_launch("rk_afm_forward");
}
