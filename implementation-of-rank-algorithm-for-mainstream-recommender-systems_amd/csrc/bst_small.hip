// Fused BST transformer block(s) + pooling at the reference script's own width: d_model 16
// (bst.py:192 hard-codes it; heads 1/2/4/8, T <= 64).  Reference: BSTTransformer.forward
// bst.py:66-91, the pooling of BSTModel.forward bst.py:224-241.
//
// At d 16 a sample's whole block is ~0.3 MFLOP over 3.2 KB of gathered rows: the per-layer path
// (five rk_linear GEMMs of K = N = 16 and the attention kernel, the sequence round-tripping
// through HBM between them, ~370 us per 4096-sample batch) is launch- and traffic-bound.  Here one
// wave owns one sample and lane t owns position t: the position's 16-wide rows (x, q, k, v,
// context, the FFN activations) live in registers, every projection is a per-lane 16 x 16
// matrix-vector product, and only K and V go through LDS (broadcast ds_read_b128: each query lane
// walks every key).  Softmax is two-pass
// (max, then exp-sum and P.V) per head on the hardware exp2 (v_exp_f32), masked keys at -inf as
// bst.py:80 (an all-masked row gives NaN as torch's softmax does).  f32 VALU throughout; the block is ~3k FMAs per lane.
//
// Weights and biases are read with uniform addresses straight from global memory, so they come in
// through the scalar cache into SGPRs (s_load), one operand of each v_fma: LDS carries only K and V.
//
// Work split: 256-thread workgroups (4 waves), persistent — each wave walks samples
// b = (blockIdx.x * 4 + wave) + k * gridDim.x * 4.
#include <cstdlib>

#include "common.h"
#include "mlp_stream.h"

namespace rk {

constexpr int kSD = 16;        // d_model
constexpr int kST = 64;        // positions (one per lane)
constexpr int kSMaxBlocks = 4;
constexpr int kSWaves = 4;

struct BstSmallW {
  const float* p[17];  // the header's order: pos, wq, bq, wk, bk, wv, bv, wo, bo, w1, b1, w2, b2, g1, be1, g2, be2
  float eps1, eps2, slope;
};

struct BstSmallArgs {
  const float* table;
  int64_t rows, ld;
  const int64_t* seq;
  int64_t ld_seq;
  int T;
  const int64_t* seq_len;
  int64_t batch;
  int nblocks;
  BstSmallW blk[kSMaxBlocks];
  float* pool_out;
  int64_t ld_pool;
  int pool_mean;
  uint32_t* flags;
};

typedef float f4s __attribute__((ext_vector_type(4)));
// read-only parameters through the constant address space: uniform loads become s_load (SGPRs)
typedef const __attribute__((address_space(4))) float cfloat;
typedef const __attribute__((address_space(4))) f4s cf4s;

// y = W x + b for one lane (W row-major [16][16], nn.Linear layout; uniform loads -> SGPRs)
__device__ __forceinline__ void matvec16(const float* Wg, const float* bg, const float (&x)[kSD], float (&y)[kSD]) {
  const cfloat* bias = (const cfloat*)bg;
#pragma unroll
  for (int o = 0; o < kSD; ++o) {
    // row o's address waits for row o - 2's result: at most two 16-float rows in SGPRs at a time
    // (the scheduler otherwise issues all 16 row loads up front and spills SGPRs to VGPR lanes)
    const float* row = Wg + o * kSD;
    if (o >= 2) asm volatile("" : "+s"(row) : "v"(y[o - 2]));
    const cfloat* W = (const cfloat*)row;
    float s = bias[o];
#pragma unroll
    for (int q = 0; q < kSD / 4; ++q) {
      const f4s w = *(const cf4s*)(W + 4 * q);
      s = fmaf(w[0], x[4 * q], s);
      s = fmaf(w[1], x[4 * q + 1], s);
      s = fmaf(w[2], x[4 * q + 2], s);
      s = fmaf(w[3], x[4 * q + 3], s);
    }
    y[o] = s;
  }
}

// LayerNorm over the lane's 16 values (biased variance, as torch.nn.LayerNorm)
__device__ __forceinline__ void layernorm16(float (&x)[kSD], const float* gg, const float* bg, float eps) {
  const cfloat* g = (const cfloat*)gg;
  const cfloat* be = (const cfloat*)bg;
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < kSD; ++i) m += x[i];
  m = m / (float)kSD;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < kSD; ++i) {
    const float d = x[i] - m;
    v = fmaf(d, d, v);
  }
  v = v / (float)kSD;
  const float r = 1.0f / sqrtf(v + eps);
#pragma unroll
  for (int i = 0; i < kSD; ++i) x[i] = (x[i] - m) * r * g[i] + be[i];
}

// One sample's blocks and pooling by one wave (lane t = position t): returns the pooled value of
// column `lane` in lanes 0..15.  Ks / Vs: the wave's [64][16] LDS slices.
template <int NH>
__device__ __forceinline__ float bst_small_sample(const BstSmallArgs& a, int64_t b, float* Ks, float* Vs, int lane) {
  constexpr int DH = kSD / NH;
  // scores in log2 units: exp(s / sqrt(dh) - max) = exp2(s * log2(e) / sqrt(dh) - max2) on v_exp_f32
  const float qscale = 1.4426950408889634f / sqrtf((float)DH);
  const int T = a.T;
  const bool pos_live = lane < T;
  const int64_t len = a.seq_len[b];
  float x[kSD];
  {
    const int64_t r = pos_live ? a.seq[b * a.ld_seq + lane] : 0;
    const bool ok = r >= 0 && r < a.rows;
    if (pos_live && !ok) flag_oob(a.flags);
    const float* src = a.table + (ok ? r : 0) * a.ld;
#pragma unroll
    for (int q = 0; q < kSD / 4; ++q) {
      const f4s v = *reinterpret_cast<const f4s*>(src + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) x[4 * q + e] = (pos_live && ok) ? v[e] : 0.f;
    }
  }
  for (int blk = 0; blk < a.nblocks; ++blk) {
    // the parameter pointers laundered per sample and block: loads through them stay inside the
    // loop (hoisted out of the sample loop, all 1.7k weights would be live in SGPRs and spill)
    BstSmallW w;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
      const float* pk = a.blk[blk].p[k];
      asm volatile("" : "+s"(pk));
      w.p[k] = pk;
    }
    w.eps1 = a.blk[blk].eps1;
    w.eps2 = a.blk[blk].eps2;
    w.slope = a.blk[blk].slope;
    // queries / keys get the position embedding, values do not (bst.py:69-71)
    float qin[kSD];
    {
      const float* pp = w.p[0] + (pos_live ? lane : 0) * kSD;
#pragma unroll
      for (int q4 = 0; q4 < kSD / 4; ++q4) {
        const f4s v = *reinterpret_cast<const f4s*>(pp + 4 * q4);
#pragma unroll
        for (int e = 0; e < 4; ++e) qin[4 * q4 + e] = x[4 * q4 + e] + (pos_live ? v[e] : 0.f);
      }
    }
    float q[kSD], t16[kSD];
    matvec16(w.p[3], w.p[4], qin, t16);  // k
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < kSD / 4; ++i)
      *reinterpret_cast<f4s*>(Ks + lane * kSD + 4 * i) = (f4s){t16[4 * i], t16[4 * i + 1], t16[4 * i + 2], t16[4 * i + 3]};
    matvec16(w.p[5], w.p[6], x, t16);  // v
#pragma unroll
    for (int i = 0; i < kSD / 4; ++i)
      *reinterpret_cast<f4s*>(Vs + lane * kSD + 4 * i) = (f4s){t16[4 * i], t16[4 * i + 1], t16[4 * i + 2], t16[4 * i + 3]};
    matvec16(w.p[1], w.p[2], qin, q);  // q
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // scores s_h[j] = q_h . k_h[j] / sqrt(dh), keys j >= len masked (-inf); two-pass softmax
    float m[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) m[h] = -INFINITY;
    for (int j = 0; j < T; ++j) {
      float k[kSD];
#pragma unroll
      for (int i = 0; i < kSD / 4; ++i) {
        const f4s v = *reinterpret_cast<const f4s*>(Ks + j * kSD + 4 * i);
        k[4 * i] = v[0], k[4 * i + 1] = v[1], k[4 * i + 2] = v[2], k[4 * i + 3] = v[3];
      }
      const bool masked = (int64_t)j >= len;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < DH; ++e) s = fmaf(q[h * DH + e], k[h * DH + e], s);
        s = masked ? -INFINITY : s * qscale;
        m[h] = fmaxf(m[h], s);
      }
    }
    float l[NH], ctx[kSD];
#pragma unroll
    for (int h = 0; h < NH; ++h) l[h] = 0.f;
#pragma unroll
    for (int i = 0; i < kSD; ++i) ctx[i] = 0.f;
    for (int j = 0; j < T; ++j) {
      float k[kSD], v[kSD];
#pragma unroll
      for (int i = 0; i < kSD / 4; ++i) {
        const f4s kv4 = *reinterpret_cast<const f4s*>(Ks + j * kSD + 4 * i);
        const f4s vv4 = *reinterpret_cast<const f4s*>(Vs + j * kSD + 4 * i);
#pragma unroll
        for (int e = 0; e < 4; ++e) k[4 * i + e] = kv4[e], v[4 * i + e] = vv4[e];
      }
      const bool masked = (int64_t)j >= len;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < DH; ++e) s = fmaf(q[h * DH + e], k[h * DH + e], s);
        s = masked ? -INFINITY : s * qscale;
        const float p = __builtin_amdgcn_exp2f(s - m[h]);
        l[h] += p;
#pragma unroll
        for (int e = 0; e < DH; ++e) ctx[h * DH + e] = fmaf(p, v[h * DH + e], ctx[h * DH + e]);
      }
    }
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const float inv = 1.0f / l[h];
#pragma unroll
      for (int e = 0; e < DH; ++e) ctx[h * DH + e] = ctx[h * DH + e] * inv;
    }
    // out1 = norm1(queries + W_o ctx) (dropout: identity in eval)
    float o[kSD];
    matvec16(w.p[7], w.p[8], ctx, o);
#pragma unroll
    for (int i = 0; i < kSD; ++i) o[i] = qin[i] + o[i];
    layernorm16(o, w.p[13], w.p[14], w.eps1);
    // out = norm2(out1 + ffn(out1)), ffn = Linear, LeakyReLU, (Dropout), Linear
    matvec16(w.p[9], w.p[10], o, t16);
    const float slope = w.slope;
#pragma unroll
    for (int i = 0; i < kSD; ++i) t16[i] = t16[i] >= 0.f ? t16[i] : t16[i] * slope;
    matvec16(w.p[11], w.p[12], t16, x);
#pragma unroll
    for (int i = 0; i < kSD; ++i) x[i] = o[i] + x[i];
    layernorm16(x, w.p[15], w.p[16], w.eps2);
    __builtin_amdgcn_wave_barrier();  // K / V are rewritten by the next block (or sample)
  }
  // pooling over all T positions (bst.py:236-241: the padded positions' outputs included)
  float pooled = 0.f;
#pragma unroll
  for (int i = 0; i < kSD; ++i) {
    const float s = wave_sum(pos_live ? x[i] : 0.f);
    pooled = lane == i ? s : pooled;
  }
  return a.pool_mean ? pooled / (float)len : pooled;
}

// ---------------------------------------------------------------------------------------------
// 4 heads (d_h = 4) on the matrix cores (round 5).  One wave per sample, the sequence in 16-position
// tiles; every activation stays in registers in one layout, L0: lane (p16 = lane & 15, grp = lane >> 4)
// holds features 4 grp .. 4 grp + 3 of position 16 pt + p16 (4 VGPRs per tile) — so head h's four
// dimensions are lane group h, register e.
//  * projections Y = X W^T + b as Y^T = W X^T on v_mfma_f32_16x16x4_f32: the weights are the A
//    operand (lane l: W[l % 16][4 (l / 16) + s] for K-step s, one float4), the activation tile the B
//    operand as it stands (K-step s contracts features {4 g + s}), the bias the initial accumulator;
//    the result is again in L0.  16 MFMAs per projection over 64 positions.
//  * scores S^T_h = K_h Q_h^T on v_mfma_f32_4x4x1f32, 16 blocks = 4 heads x 4 query quads: the B
//    operand is Q's register e (lane (4 qg + j, h)), the A operand K's register e broadcast from block
//    ABID = kg of each 4-block group (CBSZ 2: lanes 16 h + 4 kg + i = keys 4 kg + i of head h), so 16
//    instructions give lane (q, h) the 16 scores of its query and head over a key tile: softmax runs
//    in-lane (online over key tiles, exp2), no cross-lane reduction.
//  * P V on the same instruction: B = the probabilities as they stand (register (kg, i) = key
//    4 kg + i), A = V transposed within each lane quad (DPP quad_perm) and broadcast with ABID = kg;
//    the context lands in L0, ready for W_o.
//  * key tiles past the sample's length are skipped (their keys are masked: exactly zero weight);
//    LayerNorm reduces over the 4 lane groups by two cross-row swaps (v_permlane16/32_swap).
// Parameters of every block (the six 16 x 16 weights, biases, LayerNorm affines, position rows) are
// staged once per workgroup in LDS: kBmBlockFloats per block.
constexpr int kBmW = 0, kBmB = 6 * 256, kBmLN = kBmB + 6 * 16, kBmSc = kBmLN + 4 * 16, kBmPos = kBmSc + 4;
constexpr int kBmBlockFloats = kBmPos + kST * kSD;  // 2724: ..., eps1 eps2 slope pad, pos

// two accumulation chains (K-steps 0, 2 on the bias; 1, 3 from zero), added at the end: the
// dependent-MFMA latency (40 cycles) paid twice per projection instead of four times
__device__ __forceinline__ f32x4_t bm_proj(const float* W, const float* bias, f32x4_t x, int lane) {
  const f32x4_t w = *reinterpret_cast<const f32x4_t*>(W + (lane & 15) * kSD + 4 * (lane >> 4));
  f32x4_t acc = *reinterpret_cast<const f32x4_t*>(bias + 4 * (lane >> 4));
  f32x4_t acc1 = {0.f, 0.f, 0.f, 0.f};
  acc = mfma16(w[0], x[0], acc);
  acc1 = mfma16(w[1], x[1], acc1);
  acc = mfma16(w[2], x[2], acc);
  acc1 = mfma16(w[3], x[3], acc1);
  return acc + acc1;
}

template <int ABID>
__device__ __forceinline__ f32x4_t mfma4b(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 2, ABID, 0);
}

// out[i][e] = in[e][i] within each lane quad (i = lane & 3, e = register)
__device__ __forceinline__ f32x4_t quad_transpose(f32x4_t m, int lane) {
  const bool b0 = lane & 1, b1 = (lane >> 1) & 1;
  float r0 = dpp_f32<0xB1>(b0 ? m[0] : m[1]);
  float r1 = dpp_f32<0xB1>(b0 ? m[2] : m[3]);
  f32x4_t m1;
  m1[0] = b0 ? r0 : m[0];
  m1[1] = b0 ? m[1] : r0;
  m1[2] = b0 ? r1 : m[2];
  m1[3] = b0 ? m[3] : r1;
  r0 = dpp_f32<0x4E>(b1 ? m1[0] : m1[2]);
  r1 = dpp_f32<0x4E>(b1 ? m1[1] : m1[3]);
  f32x4_t m2;
  m2[0] = b1 ? r0 : m1[0];
  m2[1] = b1 ? r1 : m1[1];
  m2[2] = b1 ? m1[2] : r0;
  m2[3] = b1 ? m1[3] : r1;
  return m2;
}

// LayerNorm of each position over its 16 features (4 in-lane x the 4 lane groups), biased variance
__device__ __forceinline__ f32x4_t bm_layernorm(f32x4_t x, const float* g, const float* be, float eps, int lane) {
  float s = (x[0] + x[1]) + (x[2] + x[3]);
  s = xor32_sum(xor16_sum(s));
  const float m = s / (float)kSD;
  f32x4_t d;
  float v = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    d[r] = x[r] - m;
    v = fmaf(d[r], d[r], v);
  }
  v = xor32_sum(xor16_sum(v));
  const float rs = __builtin_amdgcn_rsqf(v / (float)kSD + eps);  // v_rsq_f32 (1 ulp), not div + sqrt
  const f32x4_t gg = *reinterpret_cast<const f32x4_t*>(g + 4 * (lane >> 4));
  const f32x4_t bb = *reinterpret_cast<const f32x4_t*>(be + 4 * (lane >> 4));
  f32x4_t y;
#pragma unroll
  for (int r = 0; r < 4; ++r) y[r] = d[r] * rs * gg[r] + bb[r];
  return y;
}

// One sample (4 heads) by one wave: blocks + pooling.  prm: the LDS parameter image of all blocks.
// Returns the pooled value of feature 4 (lane >> 4) + ((lane & 15) >> 2) in lanes with lane % 4 == 0.
__device__ __forceinline__ float bst_mfma_sample(const BstSmallArgs& a, const float* prm, int64_t b, int lane) {
  const int p16 = lane & 15, grp = lane >> 4;
  const int T = a.T;
  const int64_t len = a.seq_len[b];
  // unmasked keys (bst.py:229), wave-uniform (one sample per wave) and held in an SGPR
  const int lc = __builtin_amdgcn_readfirstlane(len <= 0 ? 0 : (len >= T ? T : (int)len));
  const int NT = (T + 15) >> 4, NKT = (lc + 15) >> 4;
  constexpr float kLog2e = 1.4426950408889634f;
  const float qscale = kLog2e / 2.0f;  // log2(e) / sqrt(d_h), d_h = 4
  f32x4_t x[4];
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    x[pt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int p = 16 * pt + p16;
    if (pt < NT && p < T) {
      const int64_t r = a.seq[b * a.ld_seq + p];
      if (r >= 0 && r < a.rows)
        x[pt] = *reinterpret_cast<const f32x4_t*>(a.table + r * a.ld + 4 * grp);
      else
        flag_oob(a.flags);
    }
  }
  for (int blk = 0; blk < a.nblocks; ++blk) {
    const float* P = prm + blk * kBmBlockFloats;
    const float* Wq = P + kBmW;
    const float* Wk = Wq + 256;
    const float* Wv = Wk + 256;
    const float* Wo = Wv + 256;
    const float* W1 = Wo + 256;
    const float* W2 = W1 + 256;
    const float* B = P + kBmB;
    const float* LN = P + kBmLN;
    // queries / keys get the position embedding, values do not (bst.py:69-71); formed where used
    // (a tile's x is overwritten only after its last use in this block)
    auto qin = [&](int pt) {
      f32x4_t v = x[pt];
      const int p = 16 * pt + p16;
      if (p < T) v += *reinterpret_cast<const f32x4_t*>(P + kBmPos + p * kSD + 4 * grp);
      return v;
    };
    f32x4_t K[4], Vq[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      if (kt < NKT) {
        K[kt] = bm_proj(Wk, B + 16, qin(kt), lane);
        Vq[kt] = quad_transpose(bm_proj(Wv, B + 32, x[kt], lane), lane);
      }
    }
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      if (qt >= NT) break;
      // the parameter loads stay inside the tile (hoisted, the 4 projections' weights, biases and
      // LayerNorm affines would hold 48 VGPRs across the tile loop and spill)
      asm volatile("" ::: "memory");
      const f32x4_t q = bm_proj(Wq, B, qin(qt), lane);
      float m_run = -INFINITY, l_run = 0.f;
      f32x4_t o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        if (kt >= NKT) break;
        f32x4_t sc[4];
#pragma unroll
        for (int kg = 0; kg < 4; ++kg) sc[kg] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sc[0] = mfma4b<0>(K[kt][e], q[e], sc[0]);
          sc[1] = mfma4b<1>(K[kt][e], q[e], sc[1]);
          sc[2] = mfma4b<2>(K[kt][e], q[e], sc[2]);
          sc[3] = mfma4b<3>(K[kt][e], q[e], sc[3]);
        }
        // lane (q, h) register (kg, i): key 16 kt + 4 kg + i; masked keys -inf (bst.py:80).  The
        // tile's key limit is laundered per tile: hoisted, the 64 compile-time key compares became 64
        // SGPR-pair masks spilled to VGPR lanes (two v_readlane per score)
        int klim = lc - 16 * kt;
        asm volatile("" : "+s"(klim));
        float mt = -INFINITY;
#pragma unroll
        for (int kg = 0; kg < 4; ++kg)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            sc[kg][i] = 4 * kg + i < klim ? sc[kg][i] * qscale : -INFINITY;
            mt = fmaxf(mt, sc[kg][i]);
          }
        const float m_new = fmaxf(m_run, mt);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        float ls = 0.f;
#pragma unroll
        for (int kg = 0; kg < 4; ++kg)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            sc[kg][i] = __builtin_amdgcn_exp2f(sc[kg][i] - m_new);
            ls += sc[kg][i];
          }
        l_run = fmaf(l_run, alpha, ls);
        m_run = m_new;
        o *= alpha;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o = mfma4b<0>(Vq[kt][i], sc[0][i], o);
          o = mfma4b<1>(Vq[kt][i], sc[1][i], o);
          o = mfma4b<2>(Vq[kt][i], sc[2][i], o);
          o = mfma4b<3>(Vq[kt][i], sc[3][i], o);
        }
      }
      // context (an all-masked row gives 0 * inf = NaN, as torch's softmax over -inf)
      o *= __builtin_amdgcn_rcpf(l_run);  // v_rcp_f32 (1 ulp); rcp(0) = inf keeps the NaN
      // out1 = norm1(queries + W_o ctx); out = norm2(out1 + W2 LeakyReLU(W1 out1)) (bst.py:85-90)
      f32x4_t o1 = bm_proj(Wo, B + 48, o, lane) + qin(qt);
      o1 = bm_layernorm(o1, LN, LN + 16, P[kBmSc], lane);
      f32x4_t f = bm_proj(W1, B + 64, o1, lane);
      const float slope = P[kBmSc + 2];
#pragma unroll
      for (int r = 0; r < 4; ++r) f[r] = f[r] >= 0.f ? f[r] : f[r] * slope;
      f = bm_proj(W2, B + 80, f, lane) + o1;
      x[qt] = bm_layernorm(f, LN + 32, LN + 48, P[kBmSc + 1], lane);
    }
  }
  // pooling over the T positions (bst.py:236-241: the padded positions' outputs included)
  float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int pt = 0; pt < 4; ++pt) {
    const bool on = pt < NT && 16 * pt + p16 < T;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += on ? x[pt][r] : 0.f;
  }
  const float pooled = row16_transpose_sum<4>(v, p16);
  return a.pool_mean ? pooled / (float)len : pooled;
}

// stage every block's parameters into the LDS image (all threads of the workgroup); static
// indexing of the argument block (a runtime-indexed kernel-argument array is copied out whole)
__device__ __forceinline__ void bst_mfma_stage(const BstSmallArgs& a, float* prm, int tid, int nthreads) {
  // image order: wq wk wv wo w1 w2 | bq bk bv bo b1 b2 | g1 be1 g2 be2 | pos[T][16]
  constexpr int kSrc[16] = {1, 3, 5, 7, 9, 11, 2, 4, 6, 8, 10, 12, 13, 14, 15, 16};
  const int npos = a.T * kSD;
#pragma unroll
  for (int blk = 0; blk < kSMaxBlocks; ++blk) {
    if (blk < a.nblocks) {
      float* dst = prm + blk * kBmBlockFloats;
      static_for<0, 16>([&](auto KI) {
        constexpr int k = KI;
        constexpr int n = k < 6 ? 256 : 16;
        constexpr int off = k < 6 ? 256 * k : kBmB + 16 * (k - 6);
        const float* src = a.blk[blk].p[kSrc[k]];
        for (int i = tid; i < n; i += nthreads) dst[off + i] = src[i];
      });
      const float* pos = a.blk[blk].p[0];
      for (int i = tid; i < npos; i += nthreads) dst[kBmPos + i] = pos[i];
      if (tid == 0) {
        dst[kBmSc] = a.blk[blk].eps1;
        dst[kBmSc + 1] = a.blk[blk].eps2;
        dst[kBmSc + 2] = a.blk[blk].slope;
      }
    }
  }
}

// rk_bst_forward_blocks at d 16, 4 heads: the blocks + pooling only (bench roofline launch), 16 waves
// per workgroup (the parameter image staged once per CU), persistent over the samples
constexpr int kBmWaves = 16;
__global__ __launch_bounds__(kBmWaves * 64) void bst_mfma_kernel(BstSmallArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  bst_mfma_stage(a, sm, tid, kBmWaves * 64);
  __syncthreads();
  for (int64_t b = (int64_t)blockIdx.x * kBmWaves + wave; b < a.batch; b += (int64_t)gridDim.x * kBmWaves) {
    const float v = bst_mfma_sample(a, sm, b, lane);
    if ((lane & 3) == 0) a.pool_out[b * a.ld_pool + 4 * (lane >> 4) + ((lane & 15) >> 2)] = v;
  }
}

template <int NH>
__global__ __launch_bounds__(kSWaves * 64, 4) void bst_small_kernel(BstSmallArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* const kv = sm + wave * 2 * kST * kSD;  // this wave's K [64][16], V [64][16]
  for (int64_t b = (int64_t)blockIdx.x * kSWaves + wave; b < a.batch; b += (int64_t)gridDim.x * kSWaves) {
    const float v = bst_small_sample<NH>(a, b, kv, kv + kST * kSD, lane);
    if (lane < kSD) a.pool_out[b * a.ld_pool + lane] = v;
  }
}

// The whole BSTModel eval forward at d_model 16 in one launch (bst.py:216-247): per 16-sample
// workgroup, wave w gathers sample m0 + w's DNN-row columns [dense | category embeddings] into LDS
// (bst.py:218-222), runs its transformer blocks and pooling (bst_small_sample, K / V in the wave's
// LDS slices) and writes the pooled 16 columns after them (bst.py:238-243); then the DNN tail and
// its output layer + sigmoid (bst.py:245-246) on the streamed plan over the 16 LDS rows.  The K / V
// slices alias phase B's second activation buffer: phase B writes it only after the barrier that
// opens it.  Replaces rk_concat_gather + rk_bst_forward_blocks + rk_mlp_forward (three launches and
// the DNN row's round trip through HBM).
constexpr int kBfSegs = 8;
constexpr int kBfCols = 128;  // row columns [0, width + 16) within one 128-wide K plan
struct BstFwdArgs {
  BstSmallArgs s;  // blocks, sequence, flags (pool_out unused)
  rk_segment segs[kBfSegs];
  uint8_t col_seg[kBfCols], col_off[kBfCols];  // row column -> (segment, offset); 255: zero
  int width;                                   // pooled columns at [width, width + 16)
  rk_mlp_layer L[RK_MLP_MAX_LAYERS];
  rk_epilogue head;
  int ld0, ld1, off1;  // LDS (floats): buf0 [16][ld0]; at off1 buf1 [16][ld1] / the K, V slices
  int off_p;           // 4 heads on MFMA: the blocks' parameter image (kBmBlockFloats per block)
};
static_assert(sizeof(BstFwdArgs) <= 4096, "kernel arguments beyond 4 KiB");

// P: the DNN tail's plan — StreamPlanK80 when the row (+ pooled columns) fits 80 columns (the
// reference's 66: layer 0 streams 5 of its image's 8 K-chunks, the other 3 multiply zero columns)
template <int NH, class P>
__global__ __launch_bounds__(kMlpThreads) void bst_small_fwd_kernel(BstFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * kMlpRows;
  const int rows = (int)min<int64_t>(kMlpRows, a.s.batch - m0);
  const int64_t b = m0 + wave;
  const bool live = wave < rows;
  float* const buf0 = sm;
  float* const buf1 = sm + a.off1;
  float* const kv = buf1 + wave * 2 * kST * kSD;
  float* const row = buf0 + wave * a.ld0;
  // the row's gathered columns (zero past `width` and for a sample past the batch)
#pragma unroll
  for (int i = 0; i < kBfCols / 64; ++i) {
    const int c = lane + 64 * i;
    float v = 0.f;
    const int sg = live && c < a.width ? a.col_seg[c] : 255;
    if (sg != 255) {
      const rk_segment& g = a.segs[sg];
      int64_t r = b;
      if (g.idx) {
        r = g.idx[b * g.idx_stride];
        if (r < 0 || r >= g.rows) {
          flag_oob(a.s.flags);
          r = -1;
        }
      }
      if (r >= 0) v = g.src[r * g.src_ld + a.col_off[c]];
    }
    row[c] = v;
  }
  const float pooled = live ? bst_small_sample<NH>(a.s, b, kv, kv + kST * kSD, lane) : 0.f;
  if (lane < kSD) row[a.width + lane] = pooled;
  mlp_stream_rows<P, kEpiRegs>(a.L, buf0, a.ld0, buf1, a.ld1, nullptr, m0, rows, a.head, tid);
}

// The same forward with 4 heads on the matrix cores (bst_mfma_sample): no K / V slices in LDS; the
// blocks' parameter image after buf1.
template <class P>
__global__ __launch_bounds__(kMlpThreads) void bst_mfma_fwd_kernel(BstFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * kMlpRows;
  const int rows = (int)min<int64_t>(kMlpRows, a.s.batch - m0);
  const int64_t b = m0 + wave;
  const bool live = wave < rows;
  float* const buf0 = sm;
  float* const buf1 = sm + a.off1;
  float* const prm = sm + a.off_p;
  float* const row = buf0 + wave * a.ld0;
  bst_mfma_stage(a.s, prm, tid, kMlpThreads);
#pragma unroll
  for (int i = 0; i < kBfCols / 64; ++i) {
    const int c = lane + 64 * i;
    float v = 0.f;
    const int sg = live && c < a.width ? a.col_seg[c] : 255;
    if (sg != 255) {
      const rk_segment& g = a.segs[sg];
      int64_t r = b;
      if (g.idx) {
        r = g.idx[b * g.idx_stride];
        if (r < 0 || r >= g.rows) {
          flag_oob(a.s.flags);
          r = -1;
        }
      }
      if (r >= 0) v = g.src[r * g.src_ld + a.col_off[c]];
    }
    row[c] = v;
  }
  __syncthreads();  // the parameter image
  if (live) {
    const float pooled = bst_mfma_sample(a.s, prm, b, lane);
    if ((lane & 3) == 0) row[a.width + 4 * (lane >> 4) + ((lane & 15) >> 2)] = pooled;
  } else if (lane < kSD) {
    row[a.width + lane] = 0.f;
  }
  mlp_stream_rows<P, kEpiRegs>(a.L, buf0, a.ld0, buf1, a.ld1, nullptr, m0, rows, a.head, tid);
}

static bool bst_use_mfma(int heads) {
  if (heads != 4) return false;
  const char* e = getenv("RANKOPS_BST_MFMA");  // 0: the VALU kernels (A/B timing)
  return !(e && e[0] == '0');
}

RK_API int rk_bst_small_forward(const rk_segment* row_segs, int32_t nseg, int32_t width, const float* table,
                                int64_t table_rows, int64_t ld_table, const int64_t* seq, int64_t ld_seq, int32_t T,
                                const int64_t* seq_len, int64_t batch, int32_t heads, int32_t nblocks,
                                const float* const* block_params, const float* block_scalars, int32_t pool_mean,
                                const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head, void* stream) {
  if (heads != 1 && heads != 2 && heads != 4 && heads != 8)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_small_forward: %d heads (1, 2, 4 or 8)", heads);
  if (T <= 0 || T > kST) return fail(RK_ERR_UNSUPPORTED, "rk_bst_small_forward: T=%d outside [1, %d]", T, kST);
  if (nblocks <= 0 || nblocks > kSMaxBlocks)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_small_forward: %d blocks (1..%d)", nblocks, kSMaxBlocks);
  if (!row_segs || nseg <= 0 || nseg > kBfSegs || width <= 0 || width + kSD > kBfCols)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_small_forward: %d row segments over %d columns", nseg, width);
  if (!table || !seq || !seq_len || !block_params || !block_scalars || !head || !head->head_w || ld_table % 4 ||
      ((uintptr_t)table & 15u) || ld_seq < T || table_rows <= 0 || batch < 0)
    return fail(RK_ERR_INVALID, "rk_bst_small_forward: bad arguments");
  const int K0 = width + kSD;
  if (stream_plan_for(layers, nlayers, K0) != kStreamK128)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_small_forward: the DNN tail has no compiled plan over %d columns", K0);
  BstFwdArgs a = {};
  int need0 = 0, need1 = 0;
  a.head = *head;
  if (int e = mlp_validate(layers, nlayers, K0, a.head, &need0, &need1, "rk_bst_small_forward")) return e;
  for (int l = 0; l < nlayers; ++l) a.L[l] = layers[l];
  for (int c = 0; c < kBfCols; ++c) {  // the last covering segment wins (rk_concat_gather)
    a.col_seg[c] = 255;
    a.col_off[c] = 0;
  }
  for (int sg = 0; sg < nseg; ++sg) {
    const rk_segment& g = row_segs[sg];
    if (!g.src || g.dim <= 0 || g.out_col < 0 || g.out_col + g.dim > width || (g.idx && g.rows <= 0))
      return fail(RK_ERR_INVALID, "rk_bst_small_forward: row segment %d invalid", sg);
    a.segs[sg] = g;
    for (int c = g.out_col; c < g.out_col + g.dim; ++c) {
      a.col_seg[c] = (uint8_t)sg;
      a.col_off[c] = (uint8_t)(c - g.out_col);
    }
  }
  a.width = width;
  BstSmallArgs& s = a.s;
  s.table = table;
  s.rows = table_rows;
  s.ld = ld_table;
  s.seq = seq;
  s.ld_seq = ld_seq;
  s.T = T;
  s.seq_len = seq_len;
  s.batch = batch;
  s.nblocks = nblocks;
  for (int i = 0; i < nblocks; ++i) {
    for (int k = 0; k < 17; ++k) {
      const float* p = block_params[17 * i + k];
      if (!p || ((uintptr_t)p & 15u))
        return fail(RK_ERR_INVALID, "rk_bst_small_forward: block %d parameter %d null or misaligned", i, k);
      s.blk[i].p[k] = p;
    }
    s.blk[i].eps1 = block_scalars[3 * i];
    s.blk[i].eps2 = block_scalars[3 * i + 1];
    s.blk[i].slope = block_scalars[3 * i + 2];
  }
  s.pool_mean = pool_mean;
  s.flags = device_flags();
  a.ld0 = need0 + kMlpLdPad;
  a.ld1 = need1 + kMlpLdPad;
  a.off1 = kMlpRows * a.ld0;
  const bool mfma = bst_use_mfma(heads);
  size_t shm;
  if (mfma) {
    a.off_p = (a.off1 + kMlpRows * a.ld1 + 3) / 4 * 4;
    shm = ((size_t)a.off_p + (size_t)nblocks * kBmBlockFloats) * sizeof(float);
  } else {
    const size_t region = std::max<size_t>((size_t)kMlpWaves * 2 * kST * kSD, (size_t)kMlpRows * a.ld1);
    shm = ((size_t)a.off1 + region) * sizeof(float);
  }
  if (shm > 160 * 1024 - kStreamStaticLds)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_small_forward: %zu B of LDS needed", shm);
  if (batch == 0) return RK_OK;
  const int64_t blocks = (batch + kMlpRows - 1) / kMlpRows;
  if (blocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_bst_small_forward: batch too large");
  auto go = [&](auto kern) {
    raise_lds_limit((const void*)kern, 160 * 1024);
    kern<<<(unsigned)blocks, kMlpThreads, shm, (hipStream_t)stream>>>(a);
  };
  // the tail's K chunks: 5 when the row fits 80 columns (RANKOPS_BST_K80=0: all 8, A/B)
  static const bool k80_on = [] {
    const char* e = getenv("RANKOPS_BST_K80");
    return !(e && e[0] == '0');
  }();
  const bool k80 = k80_on && K0 <= StreamPlanK80::KC0 * 16;
  auto launch = [&](auto plan) {
    using P = decltype(plan);
    if (mfma) return go(bst_mfma_fwd_kernel<P>);
    switch (heads) {
      case 1: go(bst_small_fwd_kernel<1, P>); break;
      case 2: go(bst_small_fwd_kernel<2, P>); break;
      case 4: go(bst_small_fwd_kernel<4, P>); break;
      default: go(bst_small_fwd_kernel<8, P>); break;
    }
  };
  if (k80)
    launch(StreamPlanK80{});
  else
    launch(StreamPlanK128{});
  return check_launch("rk_bst_small_forward");
}

int bst_small_forward(const float* table, int64_t table_rows, int64_t ld_table, const int64_t* seq, int64_t ld_seq,
                      int32_t T, const int64_t* seq_len, int64_t batch, int32_t heads, int32_t nblocks,
                      const float* const* block_params, const float* block_scalars, float* pool_out, int64_t ld_pool,
                      int32_t pool_mean, hipStream_t st) {
  if (heads != 1 && heads != 2 && heads != 4 && heads != 8)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_forward_blocks: d_model 16 with %d heads (1, 2, 4 or 8)", heads);
  if (T <= 0 || T > kST) return fail(RK_ERR_UNSUPPORTED, "rk_bst_forward_blocks: T=%d outside [1, %d]", T, kST);
  if (nblocks <= 0 || nblocks > kSMaxBlocks)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_forward_blocks: %d blocks (max %d)", nblocks, kSMaxBlocks);
  if (!table || !seq || !seq_len || !block_params || !block_scalars || !pool_out || ld_table % 4 ||
      ((uintptr_t)table & 15u) || ld_seq < T || ld_pool < kSD || table_rows <= 0)
    return fail(RK_ERR_INVALID, "rk_bst_forward_blocks: bad arguments");
  BstSmallArgs a = {};
  a.table = table;
  a.rows = table_rows;
  a.ld = ld_table;
  a.seq = seq;
  a.ld_seq = ld_seq;
  a.T = T;
  a.seq_len = seq_len;
  a.batch = batch;
  a.nblocks = nblocks;
  for (int i = 0; i < nblocks; ++i) {
    for (int k = 0; k < 17; ++k) {
      const float* p = block_params[17 * i + k];
      if (!p || ((uintptr_t)p & 15u))
        return fail(RK_ERR_INVALID, "rk_bst_forward_blocks: block %d parameter %d null or misaligned", i, k);
      a.blk[i].p[k] = p;
    }
    a.blk[i].eps1 = block_scalars[3 * i];
    a.blk[i].eps2 = block_scalars[3 * i + 1];
    a.blk[i].slope = block_scalars[3 * i + 2];
  }
  a.pool_out = pool_out;
  a.ld_pool = ld_pool;
  a.pool_mean = pool_mean;
  a.flags = device_flags();
  if (batch <= 0) return batch == 0 ? RK_OK : fail(RK_ERR_INVALID, "rk_bst_forward_blocks: negative batch");
  if (bst_use_mfma(heads)) {
    const size_t pshm = (size_t)nblocks * kBmBlockFloats * sizeof(float);
    const int64_t need = (batch + kBmWaves - 1) / kBmWaves;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(need, (int64_t)num_cus()));
    bst_mfma_kernel<<<grid, kBmWaves * 64, pshm, st>>>(a);
    return check_launch("rk_bst_forward_blocks (d_model 16, MFMA)");
  }
  const size_t shm = (size_t)(kSWaves * 2 * kST * kSD) * sizeof(float);
  const int per_cu = std::max<int>(1, std::min<int>(8, (int)((160 * 1024) / shm)));
  const int64_t need = (batch + kSWaves - 1) / kSWaves;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(need, (int64_t)num_cus() * per_cu));
  switch (heads) {
    case 1: bst_small_kernel<1><<<grid, kSWaves * 64, shm, st>>>(a); break;
    case 2: bst_small_kernel<2><<<grid, kSWaves * 64, shm, st>>>(a); break;
    case 4: bst_small_kernel<4><<<grid, kSWaves * 64, shm, st>>>(a); break;
    default: bst_small_kernel<8><<<grid, kSWaves * 64, shm, st>>>(a); break;
  }
  return check_launch("rk_bst_forward_blocks (d_model 16)");
}

}  // namespace rk
